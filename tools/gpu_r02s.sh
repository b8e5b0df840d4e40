#!/bin/bash
# final-tree evidence (tools/gpu_r02r.sh), then cross-attention GPU times without the host enqueue
# (graph mode): production launch shape vs 2-wave workgroups for the small grids (variant 50)
set -u
export TMPDIR=/tmp
bash tools/gpu_r02r.sh || exit $?
out=gpurun_out/r02r
CROSS_BENCH_GRAPH=1 timeout -k 10 180 python3 -u tools/cross_bench.py 40 > $out/cross_bench_graph.log 2>&1 || { tail -5 $out/cross_bench_graph.log; exit 1; }
grep geom $out/cross_bench_graph.log
CROSS_BENCH_GRAPH=1 P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=50 timeout -k 10 180 python3 -u tools/cross_bench.py 40 > $out/cross_bench_graph_w2.log 2>&1 || { tail -5 $out/cross_bench_graph_w2.log; exit 1; }
grep geom $out/cross_bench_graph_w2.log
