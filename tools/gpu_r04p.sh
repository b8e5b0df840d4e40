set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/${TAG:-r04p}
export P2P_EXPERIMENTS_LIB=1
i=0
for v in ${VARIANTS:-0 137 0 137}; do
  i=$((i+1))
  P2P_SELF_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG:-r04p}/prof_$i -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG:-r04p}/prof_$i.log 2>&1 || { tail gpurun_out/${TAG:-r04p}/prof_$i.log; exit 1; }
  python3 tools/rocpd_summary.py $(find gpurun_out/${TAG:-r04p}/prof_$i -name "*.db" | head -1) > gpurun_out/${TAG:-r04p}/summary_${i}_v$v.txt
  rm -rf gpurun_out/${TAG:-r04p}/prof_$i
  echo "== run $i variant $v"; grep "cross_attn_kernel\|cross_group\|self_ring\|self_split" gpurun_out/${TAG:-r04p}/summary_${i}_v$v.txt | grep wgs | cut -c1-135
done
