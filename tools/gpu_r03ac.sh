set -o pipefail
mkdir -p gpurun_out/r03ac
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r03ac/bench_default.log 2>&1 || { tail -20 gpurun_out/r03ac/bench_default.log; exit 1; }
grep '^{' gpurun_out/r03ac/bench_default.log | tail -1 > gpurun_out/r03ac/bench_default.json
timeout -k 10 400 python -u bench.py --no-cpu-baseline --store-self --steps 2 > gpurun_out/r03ac/bench_store_self.log 2>&1 || { tail -20 gpurun_out/r03ac/bench_store_self.log; exit 1; }
grep '^{' gpurun_out/r03ac/bench_store_self.log | tail -1 > gpurun_out/r03ac/bench_store_self.json
timeout -k 10 600 python -u bench.py --no-cpu-baseline --seeds 64 --groups-per-call 8 > gpurun_out/r03ac/bench_seeds64.log 2>&1 || { tail -20 gpurun_out/r03ac/bench_seeds64.log; exit 1; }
grep '^{' gpurun_out/r03ac/bench_seeds64.log | tail -1 > gpurun_out/r03ac/bench_seeds64.json
python3 -c "
import json
for f in ('bench_default','bench_store_self','bench_seeds64'):
    d=json.load(open('gpurun_out/r03ac/'+f+'.json'))
    print(f, round(d['value'],4), round(d['roofline']['frac'],4), [(x['kernel'][:22], round(x['avg_launch_ms']*1e3,2), round(x['frac'],4)) for x in d['roofline_hbm']])
"
