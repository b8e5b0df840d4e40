# in-pipeline A/B of d = 80 self-attention shapes (experiments lib): bench.py per variant
set -u
export TMPDIR=/tmp
export P2P_EXPERIMENTS_LIB=1
for v in ${VARIANTS:-0 102 103 104 105 106 102}; do
  P2P_SELF_VARIANT=$v bash tools/gpu.sh r05l_v$v bench:"--gpus 1 --steps 4 --warmup 2 --no-cpu-baseline" > /dev/null || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/r05l_v$v/bench.json'))
print('variant $v', round(d['value'],4), [(g['geometry'], round(g['avg_launch_ms']*1e3,1)) for g in d['roofline_attn_total']['by_geometry'] if g['geometry'].startswith('self:P1024')])"
done
