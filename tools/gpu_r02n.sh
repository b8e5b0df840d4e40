#!/bin/bash
# f16 dense mapper + partial-block masking in the cross kernel: timings, the cross/controller/
# forward/group/bench-config parity tests, then rocprofv3 of two timed bench groups and the PMC
# passes of the dominant kernel (profiles/r02b).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/cross_bench.py 50 > gpurun_out/cross_bench_r02n.log 2>&1 || { tail -5 gpurun_out/cross_bench_r02n.log; exit 1; }
grep geom gpurun_out/cross_bench_r02n.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_controllers.py tests/test_gpu_forward.py tests/test_gpu_groups.py \
  tests/test_gpu_blend_fold.py tests/test_gpu_bench_config.py tests/test_capi.py > gpurun_out/r02n_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r02n_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh r02o 0 42 43 0 42 || exit $?
bash tools/gpu_r02_prof.sh r02n
