#!/bin/bash
# Same-box A/B of a compile-flag change: the production library (A) against the experiments
# library (B, built with `make EXPERIMENTS=1 EXTRA_CXXFLAGS=...`, P2P_SELF_VARIANT unset = the
# production kernels), A B A B, each a rocprofv3 --kernel-trace --stats run of bench.py.
# Push with tools/gpu_ab.sh (EXTRA_CXXFLAGS in the env so its make keeps the flags):
#   EXTRA_CXXFLAGS=-fno-slp-vectorize tools/gpu_ab.sh --timeout 900 -- 'bash tools/gpu_flag_ab.sh r05slp'
# With VA / VB set, both sides run the experiments library, A under P2P_SELF_VARIANT=$VA and B
# under $VB (a variant A/B without the production-vs-experiments build difference):
#   tools/gpu_ab.sh --timeout 900 -- 'VA=0 VB=201 bash tools/gpu_flag_ab.sh r05v201'
set -u
export TMPDIR=/tmp
tag=${1:-flagab}
args=${BENCH_ARGS:---gpus 1 --steps 3 --warmup 1 --no-cpu-baseline}
out=gpurun_out/$tag
mkdir -p "$out"
i=0
for lib in A B A B; do
  i=$((i + 1))
  d="$out/prof_${lib}$i"
  if [ -n "${VA:-}" ]; then
    export P2P_EXPERIMENTS_LIB=1
    if [ $lib = A ]; then export P2P_SELF_VARIANT=$VA; else export P2P_SELF_VARIANT=$VB; fi
  elif [ $lib = B ]; then export P2P_EXPERIMENTS_LIB=1; else unset P2P_EXPERIMENTS_LIB; fi
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$d" -o run -- python3 -u bench.py $args > "$out/run_${lib}$i.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc ($lib$i)"; tail -30 "$out/run_${lib}$i.log"; exit $rc; fi
  db=$(find "$d" -name "*.db" | head -1)
  python3 tools/rocpd_summary.py "$db" > "$out/rocprof_${lib}$i.txt"
  rm -rf "$d"
  echo "== $lib$i  $(grep '^{' "$out/run_${lib}$i.log" | python3 -c 'import json,sys; print(round(json.loads(sys.stdin.read())["value"], 4))')"
  sed -n '/hot path/,$p' "$out/rocprof_${lib}$i.txt" | head -16
done
exit 0
