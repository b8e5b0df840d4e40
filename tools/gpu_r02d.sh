#!/bin/bash
# Round 2: G1 kernel schedule A/B (16x16 PV, pipelined variants) -- correctness + timing.
set -u
export TMPDIR=/tmp
out=gpurun_out/r02d
mkdir -p $out
for v in 0 10 12 15 13 14 11 0 12; do
  echo "== G1 A/B variant $v"
  P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v timeout -k 10 120 python -u tools/g1_ab.py >> $out/g1_ab.log 2>&1; rc=$?
  tail -1 $out/g1_ab.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
