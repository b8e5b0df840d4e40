#!/bin/bash
# Other BASELINE configs on one MI355X: configs[2]-shaped batches (G = 8 groups per U-Net call) and a
# configs[3] seed sweep (--seeds, all seeds timed, 8 groups per call), both bf16 U-Net + bf16 kernels.
set -u
export TMPDIR=/tmp
out=gpurun_out/r02_configs
mkdir -p $out
echo "== G=8 groups per call"
timeout -k 10 600 python -u bench.py --groups-per-call 8 --steps 1 --warmup 1 --no-cpu-baseline > $out/bench_groups8.log 2>&1; rc=$?
tail -1 $out/bench_groups8.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
echo "== seed sweep (configs[3] mode), 64 seeds"
timeout -k 10 900 python -u bench.py --seeds 64 --groups-per-call 8 --warmup 1 --no-cpu-baseline > $out/bench_seeds64.log 2>&1; rc=$?
tail -1 $out/bench_seeds64.log | cut -c1-400
exit $rc
