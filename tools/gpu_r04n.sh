set -u
export TMPDIR=/tmp
bash tools/gpu_pmc.sh g1_r04n 20 || exit 1
bash tools/gpu.sh r04n bench:"--gpus 1 --steps 20 --warmup 5" prof:"--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline" || exit 1
