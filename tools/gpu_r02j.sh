#!/bin/bash
# F16 self-attention form vs the bf16 form (A/B, experiments build), then the kernel parity tests.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_ab.sh r02j 0 40 0 40 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_controllers.py tests/test_gpu_fullsize.py > gpurun_out/r02j_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r02j_tests.log; exit $rc
