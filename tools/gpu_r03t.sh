set -o pipefail
mkdir -p gpurun_out/r03t
bash tools/gpu.sh r03t files:tests/test_gpu_kernels.py,tests/test_gpu_blend_fold.py,tests/test_gpu_controllers.py,tests/test_gpu_groups.py || exit 1
P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=0 CROSS_BENCH_GRAPH=1 timeout -k 10 300 python -u tools/cross_bench.py > gpurun_out/r03t/cross_v0.log 2>&1 || { tail -20 gpurun_out/r03t/cross_v0.log; exit 1; }
grep '^{' gpurun_out/r03t/cross_v0.log
P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=90 timeout -k 10 200 python -u tools/cross_stamps.py > gpurun_out/r03t/cross_stamps.log 2>&1 || { tail -20 gpurun_out/r03t/cross_stamps.log; exit 1; }
grep -A2 "G2\|G3" gpurun_out/r03t/cross_stamps.log
