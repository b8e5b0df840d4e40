# self40 variants: correctness + isolated timing (tools/g1_ab.py at the variant's shape) and the
# in-pipeline bench (experiments lib)
set -u
export TMPDIR=/tmp
export P2P_EXPERIMENTS_LIB=1
TAG=${TAG:-r05v}
mkdir -p gpurun_out/$TAG
for spec in ${SPECS:-"176:4096,40" "114:1024,80"}; do
  v=${spec%%:*}; shape=${spec#*:}
  P2P_SELF_VARIANT=$v G1AB_SHAPE=$shape timeout -k 10 150 python -u tools/g1_ab.py > gpurun_out/$TAG/ab_$v.log 2>&1 || { tail -20 gpurun_out/$TAG/ab_$v.log; exit 1; }
  tail -1 gpurun_out/$TAG/ab_$v.log
done
for v in ${VARIANTS:-0 176 114 0 176 114}; do
  P2P_SELF_VARIANT=$v bash tools/gpu.sh ${TAG}_v$v bench:"--gpus 1 --steps 4 --warmup 2 --no-cpu-baseline" > /dev/null || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/${TAG}_v$v/bench.json'))
print('variant $v', round(d['value'],4), [(g['geometry'], round(g['avg_launch_ms']*1e3,1)) for g in d['roofline_attn_total']['by_geometry'] if g['geometry'].startswith('self')])"
done
