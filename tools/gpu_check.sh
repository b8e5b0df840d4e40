set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== attn bench"; timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1; rc=$?; cat gpurun_out/attn_bench.log | grep geom; echo "rc=$rc"
if [ $rc -ne 0 ]; then tail -20 gpurun_out/attn_bench.log; exit $rc; fi
echo "== gpu tests"; timeout -k 10 1000 python -m pytest tests -m gpu -q -s --timeout=900 > gpurun_out/gpu_tests.log 2>&1; rc=$?
grep -E "cosine|passed|failed|Error" gpurun_out/gpu_tests.log | tail -30
echo "tests rc=$rc"
exit $rc
