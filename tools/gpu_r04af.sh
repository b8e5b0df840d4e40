set -u
export TMPDIR=/tmp
bash tools/gpu.sh r04af tests smoke bench:"--gpus 1 --steps 20 --warmup 5" prof:"--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline" || exit 1
