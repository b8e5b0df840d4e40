#!/bin/bash
# Round evidence: GPU test suite, default bench line, rocprofv3 kernel-trace summary of the bench.
set -u
export TMPDIR=/tmp
out=gpurun_out/${1:-full}
mkdir -p $out
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?
tail -3 $out/gpu_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
echo "== bench"
timeout -k 10 900 python -u bench.py > $out/bench_default.log 2>&1; rc=$?
tail -1 $out/bench_default.log | cut -c1-600; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
echo "== rocprof"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/prof_stdout.log 2>&1; rc=$?
echo "rocprof rc=$rc"; [ $rc -ne 0 ] && { tail -5 $out/prof_stdout.log; exit $rc; }
f=$(find $out/prof -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py $f > $out/timed_group_summary.txt
gzip -f $f
ls $out/prof/*/ 2>/dev/null | head
exit 0
