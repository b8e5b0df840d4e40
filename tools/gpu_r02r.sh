#!/bin/bash
# Round-2 final-tree evidence: whole GPU suite, smoke, default bench line, the batched-groups
# line (configs[2]-shaped batch of 8 groups) and the cross-kernel component timings.
set -u
export TMPDIR=/tmp
bash tools/gpu_r02_evidence.sh r02r || exit $?
out=gpurun_out/r02r
timeout -k 10 600 python -u bench.py --groups-per-call 8 --no-cpu-baseline > $out/bench_groups8.log 2>&1 || { tail -5 $out/bench_groups8.log; exit 1; }
tail -1 $out/bench_groups8.log > $out/bench_groups8.json; cut -c1-200 $out/bench_groups8.json
timeout -k 10 120 python3 -u tools/cross_bench.py 50 > $out/cross_bench.log 2>&1 || exit 1
grep geom $out/cross_bench.log
