set -u
export TMPDIR=/tmp
bash tools/gpu.sh r04z_t bench:"--gpus 1 --steps 6 --warmup 2 --no-cpu-baseline --launch-events torch" || exit 1
bash tools/gpu.sh r04z_f bench:"--gpus 1 --steps 6 --warmup 2 --no-cpu-baseline" || exit 1
bash tools/gpu.sh r04z_t2 bench:"--gpus 1 --steps 6 --warmup 2 --no-cpu-baseline --launch-events torch" || exit 1
bash tools/gpu.sh r04z_f2 bench:"--gpus 1 --steps 6 --warmup 2 --no-cpu-baseline" || exit 1
for t in r04z_t r04z_f r04z_t2 r04z_f2; do python3 -c "
import json,sys;d=json.load(open('gpurun_out/$t/bench.json'))
print('$t', round(d['value'],4), round(d['roofline']['avg_launch_ms']*1e3,1), round(d['roofline_attn_total']['frac'],4), [(g['geometry'], round(g['avg_launch_ms']*1e3,2)) for g in d['roofline_attn_total']['by_geometry']], [round(h['avg_launch_ms']*1e3,2) for h in d['roofline_hbm']])"; done
