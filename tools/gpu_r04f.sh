set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04f
bash tools/gpu.sh r04f files:tests/test_gpu_latent.py,tests/test_gpu_blend_fold.py || exit 1
timeout -k 10 120 python -u tools/latent_bench.py > gpurun_out/r04f/latent_bench.log 2>&1 || { tail gpurun_out/r04f/latent_bench.log; exit 1; }
grep '^{' gpurun_out/r04f/latent_bench.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r04f/prof -o run -- python3 -u tools/latent_bench.py 100 > gpurun_out/r04f/latent_prof.log 2>&1 || { tail gpurun_out/r04f/latent_prof.log; exit 1; }
python3 tools/rocpd_summary.py $(find gpurun_out/r04f/prof -name "*.db" | head -1) | sed -n '/hot path/,$p' | head -6
G1AB_SHAPE=1024,80 bash tools/gpu.sh r04f_d80 ab:0,96,95,103,0 || exit 1
