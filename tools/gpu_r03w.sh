set -o pipefail
mkdir -p gpurun_out/r03w
bash tools/gpu.sh r03w files:tests/test_gpu_kernels.py,tests/test_gpu_blend_fold.py || exit 1
for v in 0 126; do
  P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v CROSS_BENCH_GRAPH=1 timeout -k 10 300 python -u tools/cross_bench.py > gpurun_out/r03w/cross_v$v.log 2>&1 || { tail -20 gpurun_out/r03w/cross_v$v.log; exit 1; }
  echo "cross v$v"; grep '^{' gpurun_out/r03w/cross_v$v.log
done
PMC_SCRIPT=tools/cross_one.py bash tools/gpu_pmc.sh r03w_cross_g1 20 edit 4096 40 > /dev/null || exit 1
grep -E "p2p.*(FETCH_SIZE|WRITE_SIZE)" gpurun_out/pmc/r03w_cross_g1_summary.txt
