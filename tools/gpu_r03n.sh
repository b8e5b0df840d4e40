set -o pipefail
mkdir -p gpurun_out/r03n
bash tools/gpu.sh r03n files:tests/test_gpu_kernels.py || exit 1
P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=123 timeout -k 10 200 python -u tools/group_stamps.py > gpurun_out/r03n/stamps.log 2>&1 || { tail -20 gpurun_out/r03n/stamps.log; exit 1; }
head -14 gpurun_out/r03n/stamps.log
for v in 0 120; do
  P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v CROSS_BENCH_GRAPH=1 timeout -k 10 300 python -u tools/cross_bench.py > gpurun_out/r03n/cross_v$v.log 2>&1 || { tail -20 gpurun_out/r03n/cross_v$v.log; exit 1; }
  echo "cross v$v"; grep '^{' gpurun_out/r03n/cross_v$v.log | head -2
done
