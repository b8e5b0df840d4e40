#!/bin/bash
# PMC passes over the dominant kernel (tools/g1_only.py), one rocprofv3 run per counter group
# (gfx950 slot limits: 8 SQ, 4 TCC -- FETCH_SIZE alone uses 3).  Output: gpurun_out/pmc/<tag>_<pass>/
# Usage: [PMC_SCRIPT=tools/x.py] tools/gpu_pmc.sh <tag> [extra args for the script (default tools/g1_only.py)]
set -u
tag=${1:-cur}; shift || true
export TMPDIR=/tmp
out=gpurun_out/pmc
mkdir -p $out
passes=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
)
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  d=$out/${tag}_p$i
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d $d -o run -- python3 ${PMC_SCRIPT:-tools/g1_only.py} "$@" > $d.log 2>&1
  rc=$?
  echo "pass $i ($p) rc=$rc"
  if [ $rc -ge 124 ]; then tail -5 $d.log; exit $rc; fi
  f=$(find $d -name "*counter_collection.csv" | head -1)
  if [ -n "$f" ]; then
    python3 tools/pmc_summary.py "$f" >> $out/${tag}_summary.txt
  else
    tail -3 $d.log
  fi
done
cat $out/${tag}_summary.txt
