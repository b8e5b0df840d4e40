set -o pipefail
mkdir -p gpurun_out/r03ad
bash tools/gpu.sh r03ad files:tests/test_gpu_forward.py,tests/test_gpu_blend_fold.py,tests/test_gpu_latent.py,tests/test_gpu_pipeline.py || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r03ad/bench_default.log 2>&1 || { tail -20 gpurun_out/r03ad/bench_default.log; exit 1; }
grep '^{' gpurun_out/r03ad/bench_default.log | tail -1 | tee gpurun_out/r03ad/bench_default.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],4), [(x['kernel'][:22], round(x['avg_launch_ms']*1e3,2), round(x['frac'],4)) for x in d['roofline_hbm']])"
