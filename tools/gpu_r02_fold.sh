#!/bin/bash
set -u
export TMPDIR=/tmp
out=gpurun_out/r02_fold
mkdir -p $out
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_bench_config.py tests/test_gpu_forward.py \
  \
  > $out/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|cosine|agreement|rel err|Error" $out/tests.log | tail -30; echo "rc=$rc"
exit $rc
