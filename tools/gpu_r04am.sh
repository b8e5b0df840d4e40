set -u
export TMPDIR=/tmp
export P2P_EXPERIMENTS_LIB=1
for v in 0 181 0 181; do
  P2P_SELF_VARIANT=$v bash tools/gpu.sh r04am_v$v bench:"--gpus 1 --seeds 24 --groups-per-call 8 --warmup 1 --no-cpu-baseline" > /dev/null || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/r04am_v$v/bench.json'))
print('variant $v', round(d['value'],4), [(g['geometry'], round(g['avg_launch_ms']*1e3,1)) for g in d['roofline_attn_total']['by_geometry'] if g['geometry'].startswith('cross')])"
done
