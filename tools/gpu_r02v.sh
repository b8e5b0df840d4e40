#!/bin/bash
# same-box, in-pipeline A/B of the d = 40 production shape: variant 0 (256-key tiles + pipelined
# sub-blocks) vs 44 (128-key tiles), experiments build, bench.py's own HIP-event roofline
set -u
export TMPDIR=/tmp
out=gpurun_out/r02v
mkdir -p $out
for v in 0 44 0 44; do
  P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 > $out/bench_v$v.log 2>&1 || { tail -5 $out/bench_v$v.log; exit 1; }
  tail -1 $out/bench_v$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('v$v', round(d['value'],4), round(r['avg_launch_ms'],5), round(r['frac'],4))" | tee -a $out/summary.txt
done
