set -u
export TMPDIR=/tmp
bash tools/gpu.sh r04b files:tests/test_gpu_latent.py,tests/test_gpu_blend_fold.py tests:"cross_group_kernel or edit_with_null" bench:"--gpus 1 --steps 20 --warmup 5" || exit 1
bash tools/gpu_pmc.sh g1_17281 || exit 1
