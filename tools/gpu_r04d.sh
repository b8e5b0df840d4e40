set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04d
bash tools/gpu.sh r04d files:tests/test_gpu_latent.py,tests/test_gpu_blend_fold.py || exit 1
timeout -k 10 120 python -u tools/latent_bench.py > gpurun_out/r04d/latent_bench.log 2>&1 || { tail gpurun_out/r04d/latent_bench.log; exit 1; }
grep '^{' gpurun_out/r04d/latent_bench.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r04d/prof -o run -- python3 -u tools/latent_bench.py 100 > gpurun_out/r04d/latent_prof.log 2>&1 || { tail gpurun_out/r04d/latent_prof.log; exit 1; }
f=$(find gpurun_out/r04d/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -12
G1AB_SHAPE=1024,80 bash tools/gpu.sh r04d_d80 ab:0,150,151,152,0 || exit 1
