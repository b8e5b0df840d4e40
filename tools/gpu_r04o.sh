set -u
export TMPDIR=/tmp
bash tools/gpu.sh r04o stamps:cross_stamps:90 || exit 1
