#!/bin/bash
# Round 2: multi-block d=40 default -- correctness (kernels + controllers) and G1 A/B.
set -u
export TMPDIR=/tmp
out=gpurun_out/r02i
mkdir -p $out
echo "== kernel + controller tests"
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_controllers.py > $out/tests.log 2>&1; rc=$?
tail -3 $out/tests.log; echo "rc=$rc"; [ $rc -ne 0 ] && exit $rc
for v in 0 16 29 27 28 0 16; do
  echo "== G1 A/B variant $v"
  P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v timeout -k 10 120 python -u tools/g1_ab.py >> $out/g1_ab.log 2>&1; rc=$?
  tail -1 $out/g1_ab.log | cut -c1-40,150-260; [ $rc -ne 0 ] && exit $rc
done
exit 0
