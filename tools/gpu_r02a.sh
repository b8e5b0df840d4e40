#!/bin/bash
# Round 2, first pass: the new parity tests, smoke, one short bench line.
set -u
export TMPDIR=/tmp
out=gpurun_out/r02a
mkdir -p $out
echo "== new gpu tests"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_controllers.py tests/test_gpu_bench_config.py -s > $out/gpu_tests_new.log 2>&1; rc=$?
grep -E "PASS|FAIL|cosine|configs\[2\]|LocalBlend masks|Error|error" $out/gpu_tests_new.log | tail -40; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
echo "== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; rc=$?
tail -2 $out/smoke.log; [ $rc -ne 0 ] && exit $rc
echo "== bench"
timeout -k 10 600 python -u bench.py --steps 2 > $out/bench.log 2>&1; rc=$?
tail -1 $out/bench.log | cut -c1-600; echo "bench rc=$rc"
exit $rc
