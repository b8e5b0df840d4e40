#!/bin/bash
# Cross-attention kernel: component timings (tools/cross_bench.py) + PMC passes at G1 plain / edit.
set -u
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/cross_bench.py 50 > gpurun_out/cross_bench.log 2>&1 || exit $?
cat gpurun_out/cross_bench.log
PMC_SCRIPT=tools/cross_one.py bash tools/gpu_pmc.sh ${1:-cross}_plain 20 plain || exit $?
PMC_SCRIPT=tools/cross_one.py bash tools/gpu_pmc.sh ${1:-cross}_edit 20 edit || exit $?
