set -u
export TMPDIR=/tmp
bash tools/gpu.sh r04ag files:tests/test_gpu_kernels.py,tests/test_gpu_bench_config.py || exit 1
