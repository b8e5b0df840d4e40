# in-pipeline A/B (experiments lib): bench.py per variant, the attention geometries' HIP-event averages
set -u
export TMPDIR=/tmp
export P2P_EXPERIMENTS_LIB=1
TAG=${TAG:-r05m}
for v in ${VARIANTS:-0 170 171 135 0}; do
  P2P_SELF_VARIANT=$v bash tools/gpu.sh ${TAG}_v$v bench:"--gpus 1 --steps 4 --warmup 2 --no-cpu-baseline" > /dev/null || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/${TAG}_v$v/bench.json'))
print('variant $v', round(d['value'],4), [(g['geometry'], round(g['avg_launch_ms']*1e3,1)) for g in d['roofline_attn_total']['by_geometry']])"
done
