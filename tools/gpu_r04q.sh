set -u
export TMPDIR=/tmp
bash tools/gpu.sh r04q files:tests/test_gpu_kernels.py,tests/test_gpu_controllers.py,tests/test_gpu_blend_fold.py,tests/test_gpu_forward.py || exit 1
