#!/bin/bash
# cross-attention component timings + the cross/self kernel parity tests
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/cross_bench.py 50 > gpurun_out/cross_bench_r02l.log 2>&1 || { tail -5 gpurun_out/cross_bench_r02l.log; exit 1; }
grep geom gpurun_out/cross_bench_r02l.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_controllers.py tests/test_gpu_forward.py tests/test_gpu_blend_fold.py > gpurun_out/r02l_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r02l_tests.log; exit $rc
