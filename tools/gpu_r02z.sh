#!/bin/bash
# final binary check: smoke, C-ABI and kernel parity tests
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02z
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02z/smoke.log 2>&1 || { tail -5 gpurun_out/r02z/smoke.log; exit 1; }
tail -1 gpurun_out/r02z/smoke.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_capi.py tests/test_gpu_kernels.py \
  > gpurun_out/r02z/tests.log 2>&1; rc=$?; tail -1 gpurun_out/r02z/tests.log; exit $rc
