#!/bin/bash
# production lib vs experiments lib, same variant (compile-flag A/B).  Usage: tools/gpu_ab2.sh <tag> <variant>
set -u
export TMPDIR=/tmp
tag=$1; v=$2
out=gpurun_out/ab_$tag
mkdir -p $out
for lib in 0 1 0 1; do
  P2P_EXPERIMENTS_LIB=$lib P2P_SELF_VARIANT=$v timeout -k 10 120 python -u tools/g1_ab.py >> $out/g1_ab.log 2>&1; rc=$?
  tail -1 $out/g1_ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('explib=$lib', d['variant'], d['ok'], d['median_ms'], d['frac_2p5'])"; [ $rc -ne 0 ] && exit $rc
done
exit 0
