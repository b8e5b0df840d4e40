set -u
export TMPDIR=/tmp
bash tools/gpu.sh r04i ab:0,17281,0,17281 tests smoke || exit 1
