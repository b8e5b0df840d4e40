set -o pipefail
mkdir -p gpurun_out/r03l
bash tools/gpu.sh r03l files:tests/test_gpu_kernels.py || exit 1
for v in 0 120 122; do
  P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v CROSS_BENCH_GRAPH=1 timeout -k 10 300 python -u tools/cross_bench.py > gpurun_out/r03l/cross_v$v.log 2>&1 || { tail -20 gpurun_out/r03l/cross_v$v.log; exit 1; }
  echo "cross v$v"; grep '^{' gpurun_out/r03l/cross_v$v.log
done
for v in 0 121; do
  P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v timeout -k 10 200 python -u tools/small_bench.py > gpurun_out/r03l/small_v$v.log 2>&1 || { tail -20 gpurun_out/r03l/small_v$v.log; exit 1; }
  grep '^{' gpurun_out/r03l/small_v$v.log
done
