set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04h
bash tools/gpu.sh r04h files:tests/test_gpu_latent.py,tests/test_gpu_blend_fold.py,tests/test_gpu_forward.py || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r04h/lprof -o run -- python3 -u tools/latent_bench.py 100 > gpurun_out/r04h/latent_prof.log 2>&1 || { tail gpurun_out/r04h/latent_prof.log; exit 1; }
grep '^{' gpurun_out/r04h/latent_prof.log
python3 tools/rocpd_summary.py $(find gpurun_out/r04h/lprof -name "*.db" | head -1) | sed -n '/hot path/,$p' | head -6
bash tools/gpu.sh r04h ab:0,160,161,162,0,161 || exit 1
