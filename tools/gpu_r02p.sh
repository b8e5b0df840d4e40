#!/bin/bash
# configs[4] null-text inversion at its stated 50 x 10 schedule vs the oracle, plus the short-schedule tests.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread -m gpu \
  tests/test_gpu_nulltext.py > gpurun_out/r02p_nulltext.log 2>&1
rc=$?; grep -E '50x10|PASS|FAIL|passed|failed' gpurun_out/r02p_nulltext.log | tail -8; exit $rc
