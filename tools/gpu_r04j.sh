set -u
export TMPDIR=/tmp
bash tools/gpu.sh r04j stamps:s40_stamps:163 || exit 1
S40_STAMPS=1024,80,4,128,2 S40_NWG=256 bash tools/gpu.sh r04j_d80 stamps:s40_stamps:164 || exit 1
