#!/bin/bash
# Full GPU suite, default bench line, and the --store-self bench line (reference AttentionStore default).
set -u
export TMPDIR=/tmp
out=gpurun_out/${1:-evidence}
mkdir -p $out
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?
tail -3 $out/gpu_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
echo "== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1; rc=$?
tail -2 $out/smoke.log; [ $rc -ne 0 ] && exit $rc
echo "== bench"
timeout -k 10 600 python -u bench.py > $out/bench_default.log 2>&1; rc=$?
tail -1 $out/bench_default.log | cut -c1-300; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
echo "== bench --store-self"
timeout -k 10 600 python -u bench.py --store-self --no-cpu-baseline > $out/bench_store_self.log 2>&1; rc=$?
tail -1 $out/bench_store_self.log | cut -c1-300; echo "bench rc=$rc"
exit $rc
