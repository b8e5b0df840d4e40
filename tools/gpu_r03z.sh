set -o pipefail
mkdir -p gpurun_out/r03z3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "key_split" > gpurun_out/r03z3/t.log 2>&1 || { tail -30 gpurun_out/r03z3/t.log; exit 1; }
tail -2 gpurun_out/r03z3/t.log
for v in 0 134; do
  P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v timeout -k 10 200 python -u tools/small_bench.py > gpurun_out/r03z3/small_v$v.log 2>&1 || { tail -20 gpurun_out/r03z3/small_v$v.log; exit 1; }
  grep '^{' gpurun_out/r03z3/small_v$v.log
done
