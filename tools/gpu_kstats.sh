#!/bin/bash
# Per-kernel durations (rocprofv3 kernel trace) of tools/g1_only.py under each P2P_SELF_VARIANT given.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/kstats
for v in "$@"; do
  P2P_SELF_VARIANT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kstats/v$v -o run -- python3 tools/g1_only.py 30 > gpurun_out/kstats/v$v.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -5 gpurun_out/kstats/v$v.log; exit $rc; fi
  f=$(find gpurun_out/kstats/v$v -name "*kernel_stats.csv" | head -1)
  echo "== variant $v"; grep -E "attn|norm" "$f" | cut -d, -f1-4 | cut -c1-200
done
