#!/bin/bash
# cross kernel: folded dense blend + short-tail softmax -- timings, then the parity tests that run it
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/cross_bench.py 50 > gpurun_out/cross_bench_r02q.log 2>&1 || { tail -5 gpurun_out/cross_bench_r02q.log; exit 1; }
grep geom gpurun_out/cross_bench_r02q.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_controllers.py tests/test_gpu_forward.py tests/test_gpu_groups.py \
  tests/test_gpu_blend_fold.py tests/test_gpu_fullsize.py tests/test_gpu_ldm.py tests/test_gpu_bench_config.py \
  tests/test_capi.py > gpurun_out/r02q_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r02q_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_r02p.sh
