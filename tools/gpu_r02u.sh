#!/bin/bash
# production d = 40 kernel now 256-key tiles + pipelined sub-blocks: kernel parity tests, the bench
# line, and the PMC passes of the new kernel (bench.py's roofline.traffic source)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02u
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_controllers.py tests/test_capi.py \
  > gpurun_out/r02u/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r02u/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r02u/bench.log 2>&1 || { tail -5 gpurun_out/r02u/bench.log; exit 1; }
tail -1 gpurun_out/r02u/bench.log > gpurun_out/r02u/bench.json; cut -c1-120 gpurun_out/r02u/bench.json
bash tools/gpu_pmc.sh r02u > gpurun_out/r02u/pmc.log 2>&1; rc=$?; tail -2 gpurun_out/r02u/pmc.log; exit $rc
