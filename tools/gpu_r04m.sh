set -u
export TMPDIR=/tmp
bash tools/gpu.sh r04m smallab:0,170,171,172,0 || exit 1
