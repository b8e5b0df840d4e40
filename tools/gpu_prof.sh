set -u
mkdir -p gpurun_out/prof_r1
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_r1 -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r1/bench_stdout.log 2>&1; rc=$?
echo "rocprof rc=$rc"
find /tmp/prof_r1 -name "*.csv" | head
for f in $(find /tmp/prof_r1 -name "*stats.csv"); do cp $f gpurun_out/prof_r1/; done
for f in $(find /tmp/prof_r1 -name "*kernel_trace.csv"); do python3 tools/trace_summary.py $f > gpurun_out/prof_r1/timed_group_summary.txt; gzip -c $f > gpurun_out/prof_r1/kernel_trace.csv.gz; done
ls -la gpurun_out/prof_r1
exit $rc
