#!/bin/bash
# HBM bytes of the kept-self-map path (tools/store_bench.py): FETCH_SIZE and WRITE_SIZE passes.
set -u
export TMPDIR=/tmp
out=gpurun_out/pmc
mkdir -p $out
tag=${1:-store}
i=0
for p in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  d=$out/${tag}_p$i
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d $d -o run -- python3 tools/store_bench.py > $d.log 2>&1
  rc=$?
  echo "pass $i ($p) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $d.log; exit $rc; fi
  f=$(find $d -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && python3 tools/pmc_summary.py "$f" | grep p2p >> $out/${tag}_summary.txt
done
cat $out/${tag}_summary.txt
