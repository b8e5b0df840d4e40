#!/bin/bash
# Round-2 evidence, part 1: the whole GPU suite, smoke, the default bench line.
set -u
export TMPDIR=/tmp
out=gpurun_out/${1:-r02ev}
mkdir -p $out
echo "== gpu tests"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?
tail -3 $out/gpu_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
echo "== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; rc=$?
tail -2 $out/smoke.log; [ $rc -ne 0 ] && exit $rc
echo "== bench"
timeout -k 10 600 python -u bench.py > $out/bench_default.log 2>&1; rc=$?
tail -1 $out/bench_default.log > $out/bench_default.json; cut -c1-400 $out/bench_default.json; echo "bench rc=$rc"
exit $rc
