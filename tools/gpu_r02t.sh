#!/bin/bash
# (1) G1 A/B: production vs PIPE + 256-key tiles (variant 43), interleaved;
# (2) configs[3] at its stated size on one GPU: 256 seeds, 8 groups per U-Net call.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02t
bash tools/gpu_ab.sh r02t 0 43 0 43 0 43 || exit $?
timeout -k 10 900 python -u bench.py --seeds 256 --groups-per-call 8 --no-cpu-baseline > gpurun_out/r02t/bench_seeds256.log 2>&1
rc=$?; tail -1 gpurun_out/r02t/bench_seeds256.log | cut -c1-300; exit $rc
