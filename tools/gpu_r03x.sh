set -o pipefail
mkdir -p gpurun_out/r03x
bash tools/gpu.sh r03x ab:0,128 || exit 1
G1AB_SHAPE=1024,80 bash tools/gpu.sh r03x80 ab:0,128 || exit 1
for v in 0 127; do
  P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v CROSS_BENCH_GRAPH=1 timeout -k 10 300 python -u tools/cross_bench.py > gpurun_out/r03x/cross_v$v.log 2>&1 || { tail -20 gpurun_out/r03x/cross_v$v.log; exit 1; }
  echo "cross v$v"; grep '^{' gpurun_out/r03x/cross_v$v.log | head -1
done
P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=128 bash tools/gpu_pmc.sh r03x_g1v128 20 > /dev/null || exit 1
grep -E "self40.*(FETCH_SIZE|WRITE_SIZE)" gpurun_out/pmc/r03x_g1v128_summary.txt
