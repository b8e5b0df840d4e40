#!/bin/bash
# Self-map store path: parity tests touching kept self maps, then the store timing tool.
set -u
export TMPDIR=/tmp
out=gpurun_out/${1:-store}
mkdir -p $out
echo "== tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_controllers.py tests/test_gpu_ldm.py -m gpu -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1; rc=$?
tail -15 $out/tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
echo "== store bench"
timeout -k 10 300 python -u tools/store_bench.py > $out/store_bench.log 2>&1; rc=$?
cat $out/store_bench.log | grep -v amdgpu.ids; echo "store rc=$rc"; [ $rc -ne 0 ] && exit $rc
echo "== kstats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o store -- python3 tools/store_bench.py > $out/prof_stdout.log 2>&1; rc=$?
echo "rocprof rc=$rc"
f=$(find $out/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-4 $f | head -12
exit $rc
