set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== gpu tests"; timeout -k 10 1000 python -m pytest tests -m gpu -q -s --timeout=900 > gpurun_out/gpu_tests.log 2>&1; rc=$?
grep -E "cosine|passed|failed|Error" gpurun_out/gpu_tests.log | tail -30
echo "tests rc=$rc"
exit $rc
