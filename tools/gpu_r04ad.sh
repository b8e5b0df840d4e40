set -u
export TMPDIR=/tmp
bash tools/gpu.sh r04ad files:tests/test_gpu_kernels.py,tests/test_gpu_groups.py,tests/test_gpu_sweep.py,tests/test_gpu_controllers.py || exit 1
TAG=r04ad VARIANTS="0 177 0 177" bash tools/gpu_r04p.sh
