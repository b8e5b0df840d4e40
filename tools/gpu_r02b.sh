#!/bin/bash
# configs[2] oracle test, smoke, one short bench line (round 2).
set -u
export TMPDIR=/tmp
out=gpurun_out/r02b
mkdir -p $out
echo "== configs[2] tests"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_bench_config.py -s -k config2 > $out/gpu_tests_cfg2.log 2>&1; rc=$?
grep -E "PASS|FAIL|cosine|configs\[2\]|Error|error" $out/gpu_tests_cfg2.log | tail -20; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
echo "== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; rc=$?
tail -2 $out/smoke.log; [ $rc -ne 0 ] && exit $rc
echo "== bench"
timeout -k 10 600 python -u bench.py --steps 2 > $out/bench.log 2>&1; rc=$?
tail -1 $out/bench.log | cut -c1-700; echo "bench rc=$rc"
exit $rc
