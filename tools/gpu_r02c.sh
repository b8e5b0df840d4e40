#!/bin/bash
# Round 2: 16x16-PV G1 kernel correctness + A/B, configs[2] oracle tests, smoke, bench.
set -u
export TMPDIR=/tmp
out=gpurun_out/r02c
mkdir -p $out
echo "== kernel tests (self attention)"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "self_attention" > $out/kernel_tests.log 2>&1; rc=$?
tail -3 $out/kernel_tests.log; echo "rc=$rc"; [ $rc -ne 0 ] && exit $rc
for v in 8 0 9 8 0; do
  echo "== G1 A/B variant $v"
  P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v timeout -k 10 120 python -u tools/g1_ab.py >> $out/g1_ab.log 2>&1; rc=$?
  tail -1 $out/g1_ab.log; [ $rc -ne 0 ] && exit $rc
done
echo "== configs[2] tests"
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_bench_config.py -s -k config2 > $out/gpu_tests_cfg2.log 2>&1; rc=$?
grep -E "PASS|FAIL|cosine|configs\[2\]|Error|error" $out/gpu_tests_cfg2.log | tail -24; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
echo "== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; rc=$?
tail -2 $out/smoke.log; [ $rc -ne 0 ] && exit $rc
echo "== bench"
timeout -k 10 600 python -u bench.py --steps 2 > $out/bench.log 2>&1; rc=$?
tail -1 $out/bench.log | cut -c1-900; echo "bench rc=$rc"
exit $rc
