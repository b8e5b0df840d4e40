#!/bin/bash
# Round-2 evidence, part 2: rocprofv3 kernel trace of two timed bench groups, PMC passes of the
# dominant kernel (tools/gpu_pmc.sh).
set -u
export TMPDIR=/tmp
tag=${1:-r02}
out=gpurun_out/prof_$tag
mkdir -p $out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$tag -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/bench_stdout.log 2>&1; rc=$?
echo "rocprof rc=$rc"; [ $rc -ne 0 ] && { tail -5 $out/bench_stdout.log; exit $rc; }
tail -1 $out/bench_stdout.log | cut -c1-300
for f in $(find /tmp/prof_$tag -name "*stats.csv"); do cp $f $out/; done
for f in $(find /tmp/prof_$tag -name "*kernel_trace.csv"); do python3 tools/trace_summary.py $f > $out/timed_group_summary.txt; done
head -12 $out/timed_group_summary.txt
bash tools/gpu_pmc.sh $tag > $out/pmc.log 2>&1; rc=$?
tail -4 $out/pmc.log; echo "pmc rc=$rc"
exit $rc
