set -o pipefail
mkdir -p gpurun_out/r03af
bash tools/gpu.sh r03af files:tests/test_gpu_kernels.py,tests/test_gpu_blend_fold.py,tests/test_gpu_controllers.py || exit 1
for v in 0 138; do
  P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v CROSS_BENCH_GRAPH=1 timeout -k 10 300 python -u tools/cross_bench.py > gpurun_out/r03af/cross_v$v.log 2>&1 || { tail -20 gpurun_out/r03af/cross_v$v.log; exit 1; }
  echo "cross v$v"; grep '^{' gpurun_out/r03af/cross_v$v.log
done
