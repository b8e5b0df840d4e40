set -o pipefail
bash tools/gpu.sh r03k files:tests/test_gpu_kernels.py,tests/test_gpu_controllers.py,tests/test_gpu_blend_fold.py,tests/test_gpu_groups.py || exit 1
CROSS_BENCH_GRAPH=1 timeout -k 10 300 python -u tools/cross_bench.py > gpurun_out/r03k/cross_new.log 2>&1 || { tail -20 gpurun_out/r03k/cross_new.log; exit 1; }
tail -4 gpurun_out/r03k/cross_new.log
P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=120 CROSS_BENCH_GRAPH=1 timeout -k 10 300 python -u tools/cross_bench.py > gpurun_out/r03k/cross_old.log 2>&1 || { tail -20 gpurun_out/r03k/cross_old.log; exit 1; }
tail -4 gpurun_out/r03k/cross_old.log
bash tools/gpu.sh r03k ab:0,104,105,106
