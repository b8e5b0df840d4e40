#!/bin/bash
# G1 kernel A/B: one process per variant (experiments build).  Usage: tools/gpu_ab.sh <tag> v1 v2 ...
set -u
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/ab_$tag
mkdir -p $out
for v in "$@"; do
  P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v timeout -k 10 120 python -u tools/g1_ab.py >> $out/g1_ab.log 2>&1; rc=$?
  tail -1 $out/g1_ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['variant'], d['ok'], d['median_ms'], d['frac_2p5'])"; [ $rc -ne 0 ] && exit $rc
done
exit 0
