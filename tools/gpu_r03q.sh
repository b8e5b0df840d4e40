set -o pipefail
mkdir -p gpurun_out/r03q
bash tools/gpu.sh r03q files:tests/test_gpu_kernels.py,tests/test_gpu_controllers.py,tests/test_gpu_blend_fold.py,tests/test_gpu_groups.py || exit 1
for v in 0 120; do
  P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v CROSS_BENCH_GRAPH=1 timeout -k 10 300 python -u tools/cross_bench.py > gpurun_out/r03q/cross_v$v.log 2>&1 || { tail -20 gpurun_out/r03q/cross_v$v.log; exit 1; }
  echo "cross v$v"; grep '^{' gpurun_out/r03q/cross_v$v.log
done
P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=90 timeout -k 10 200 python -u tools/cross_stamps.py > gpurun_out/r03q/cross_stamps.log 2>&1 || { tail -20 gpurun_out/r03q/cross_stamps.log; exit 1; }
cat gpurun_out/r03q/cross_stamps.log
for v in 0 124; do
  P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v timeout -k 10 200 python -u tools/small_bench.py > gpurun_out/r03q/small_v$v.log 2>&1 || { tail -20 gpurun_out/r03q/small_v$v.log; exit 1; }
  grep '^{' gpurun_out/r03q/small_v$v.log
done
