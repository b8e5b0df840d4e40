set -u
export TMPDIR=/tmp
bash tools/gpu.sh r04ak files:tests/test_gpu_kernels.py,tests/test_gpu_groups.py,tests/test_gpu_sweep.py,tests/test_gpu_bench_config.py bench:"--gpus 1 --seeds 64 --groups-per-call 8 --warmup 1 --no-cpu-baseline" || exit 1
