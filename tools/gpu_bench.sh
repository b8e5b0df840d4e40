set -u
mkdir -p gpurun_out/prof_r1
export TMPDIR=/tmp
echo "== gpu tests"; timeout -k 10 1000 python -m pytest tests -m gpu -q -s --timeout=900 > gpurun_out/gpu_tests.log 2>&1; rc=$?
grep -E "cosine|passed|failed" gpurun_out/gpu_tests.log | tail -5; echo "tests rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
echo "== bench (default)"; timeout -k 10 900 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; tail -1 gpurun_out/bench_default.log; echo "bench rc=$rc"
if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench_default.log; exit $rc; fi
echo "== rocprof"; timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1 -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r1/bench_stdout.log 2>&1; rc=$?
tail -1 gpurun_out/prof_r1/bench_stdout.log | cut -c1-400; echo "rocprof rc=$rc"
exit $rc
