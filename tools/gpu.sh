#!/bin/bash
# One GPU-box driver for every measurement this repo takes (run through gpurun from the repo
# root).  Each step has its own time limit, steps are chained so the first failure, time-out or
# fault ends the call, and everything lands under gpurun_out/<tag>/.
#
#   tools/gpu.sh <tag> <step> [<step> ...]
#   steps:
#     smoke                  __graft_entry__.smoke()
#     tests[:<pytest -k>]    pytest -m gpu (optionally -k filtered)
#     files:<f1,f2,..>       pytest -m gpu on the listed test files
#     ab:<v1,v2,..>          G1 A/B (tools/g1_ab.py), one process per P2P_SELF_VARIANT (experiments lib)
#     bench[:<args>]         python bench.py <args> (default: the driver's default run), JSON -> bench.json
#     prof[:<args>]          rocprofv3 --kernel-trace --stats of bench.py <args>
#     pmc:<name>:<counters>  one rocprofv3 --pmc pass (comma-separated counters) over tools/g1_only.py
#                            (G1 launches only; P2P_SELF_VARIANT / P2P_EXPERIMENTS_LIB from the env)
#     cross                  tools/cross_bench.py (cross-attention launch shapes)
#     crossab:<v1,v2,..>     tools/cross_bench.py in graph mode, one process per P2P_SELF_VARIANT (experiments lib)
#     smallab:<v1,v2,..>     tools/small_bench.py (G2/G3/G4 self-attention), one process per variant
#     stamps:<tool>:<v>      a clock-stamp tool (tools/<tool>.py) under P2P_SELF_VARIANT=v (experiments lib)
#     pmcs:<tag>:<script>:<args>  tools/gpu_pmc.sh over any launcher script (comma-separated args)
#     py:<script>[:<a1,a2,..>]  python -u <script> <a1> <a2> ..
#     g1shape:<v>:<P,d>      tools/g1_ab.py (correctness + isolated timing) of variant v at shape P,d (experiments lib)
#     variants:<v1,v2,..>[:<prefix>]  in-pipeline A/B: a short bench.py per P2P_SELF_VARIANT (experiments lib),
#                            printing the HIP-event average of every attention geometry (starting with <prefix>)
set -u
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
run() {  # run <seconds> <log> <cmd...>: time-limited, output to the log, tail on failure
  local secs=$1 log=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$log" 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; tail -30 "$log"; exit $rc; fi
}
for step in "$@"; do
  kind=${step%%:*}; arg=""; [ "$kind" != "$step" ] && arg=${step#*:}
  echo "== $step"
  case $kind in
    smoke) run 300 "$out/smoke.log" python -u -c "import __graft_entry__ as g; g.smoke()"; tail -1 "$out/smoke.log" ;;
    tests)
      if [ -n "$arg" ]; then sel=(-k "$arg"); else sel=(); fi
      run 1100 "$out/tests.log" python -u -m pytest -x -v -s --durations=25 --timeout 300 --timeout-method thread -m gpu tests "${sel[@]}"
      tail -1 "$out/tests.log" ;;
    files)
      run 1100 "$out/files.log" python -u -m pytest -x -v -s --durations=15 --timeout 300 --timeout-method thread -m gpu ${arg//,/ }
      tail -1 "$out/files.log" ;;
    ab)
      for v in ${arg//,/ }; do
        run 150 "$out/ab_$v.log" env P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v python -u tools/g1_ab.py
        tail -1 "$out/ab_$v.log" | tee -a "$out/ab.log"
      done ;;
    bench) run 900 "$out/bench.log" python -u bench.py $arg; grep '^{' "$out/bench.log" | tail -1 | tee "$out/bench.json" ;;
    prof)
      run 900 "$out/prof.log" rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python3 -u bench.py $arg
      grep '^{' "$out/prof.log" | tail -1 | tee "$out/bench_under_rocprof.json"
      find "$out/prof" -name "*kernel_stats.csv" -exec cp {} "$out/kernel_stats.csv" \;
      db=$(find "$out/prof" -name "*.db" | head -1)
      # (--split-last: the G1/G7 launches of bench.py's eager timing pass -- 3 batches x 250 by default
      # -- against the warm-up and graph replays before it)
      if [ -n "$db" ]; then python3 tools/rocpd_summary.py "$db" --split-last "${P2P_SPLIT_LAST:-750}" > "$out/rocprof_summary.txt"; sed -n '/hot path/,$p' "$out/rocprof_summary.txt" | head -14; tail -4 "$out/rocprof_summary.txt"; fi
      rm -rf "$out/prof" ;;   # (the trace database of a 20-group run is far past gpurun's 64 MiB return cap)
    pmc)
      name=${arg%%:*}; counters=${arg#*:}
      run 120 "$out/pmc_$name.log" timeout -s KILL 100 rocprofv3 --pmc ${counters//,/ } --output-format csv -d "$out/pmc_$name" -o run -- python3 -u tools/g1_only.py
      f=$(find "$out/pmc_$name" -name "*counter_collection.csv" | head -1)
      [ -n "$f" ] && python3 tools/pmc_summary.py "$f" | tee -a "$out/pmc_summary.txt" ;;
    cross) run 600 "$out/cross.log" python -u tools/cross_bench.py; tail -20 "$out/cross.log" ;;
    crossab)
      for v in ${arg//,/ }; do
        run 300 "$out/cross_v$v.log" env P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v CROSS_BENCH_GRAPH=1 python -u tools/cross_bench.py
        echo "cross v$v"; grep '^{' "$out/cross_v$v.log"
      done ;;
    smallab)
      for v in ${arg//,/ }; do
        run 200 "$out/small_v$v.log" env P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v python -u tools/small_bench.py
        grep '^{' "$out/small_v$v.log"
      done ;;
    stamps)
      tool=${arg%%:*}; v=${arg#*:}
      run 200 "$out/${tool}_v$v.log" env P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v python -u tools/$tool.py
      grep -v '^$' "$out/${tool}_v$v.log" | tail -20 ;;
    pmcs)
      ptag=${arg%%:*}; rest=${arg#*:}; script=${rest%%:*}; sargs=${rest#*:}
      PMC_SCRIPT=$script run 600 "$out/pmc_$ptag.log" bash tools/gpu_pmc.sh "$ptag" ${sargs//,/ }
      grep -E "p2p.*(FETCH_SIZE|WRITE_SIZE)" gpurun_out/pmc/${ptag}_summary.txt || true ;;
    py)
      script=${arg%%:*}; sargs=""; [ "$script" != "$arg" ] && sargs=${arg#*:}
      run 1100 "$out/py_$(basename "$script" .py).log" python -u "$script" ${sargs//,/ }
      tail -15 "$out/py_$(basename "$script" .py).log" ;;
    g1shape)
      v=${arg%%:*}; shape=${arg#*:}
      run 150 "$out/g1shape_$v.log" env P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v G1AB_SHAPE=$shape python -u tools/g1_ab.py
      tail -1 "$out/g1shape_$v.log" ;;
    variants)
      vs=${arg%%:*}; prefix=""; [ "$vs" != "$arg" ] && prefix=${arg#*:}
      for v in ${vs//,/ }; do
        run 600 "$out/variant_$v.log" env P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=$v python -u bench.py --gpus 1 --steps 4 --warmup 2 --no-cpu-baseline
        grep '^{' "$out/variant_$v.log" | tail -1 | python3 -c "
import json, sys; d = json.loads(sys.stdin.read())
print('variant $v', round(d['value'], 4), [(g['geometry'], round(g['avg_launch_ms'] * 1e3, 1))
      for g in d['roofline_attn_total']['by_geometry'] if g['geometry'].startswith('$prefix')])" | tee -a "$out/variants.txt"
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
exit 0
