set -u
export TMPDIR=/tmp
bash tools/gpu.sh r04s files:tests/test_gpu_kernels.py,tests/test_gpu_controllers.py,tests/test_gpu_blend_fold.py,tests/test_gpu_forward.py,tests/test_gpu_ldm.py,tests/test_gpu_groups.py || exit 1
