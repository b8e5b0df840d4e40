#!/bin/bash
# Round 2: NOMAX self kernel -- correctness (kernel + controller tests) and G1 A/B.
set -u
export TMPDIR=/tmp
out=gpurun_out/r02h
mkdir -p $out
echo "== kernel tests"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k self_attention \
  > $out/kernel_tests.log 2>&1; rc=$?
tail -3 $out/kernel_tests.log; echo "rc=$rc"; [ $rc -ne 0 ] && exit $rc
for v in 0 18 24 25 26 23 0 24; do
  echo "== G1 A/B variant $v"
  P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v timeout -k 10 120 python -u tools/g1_ab.py >> $out/g1_ab.log 2>&1; rc=$?
  tail -1 $out/g1_ab.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
