set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04g
timeout -k 10 120 python -u tools/latent_bench.py > gpurun_out/r04g/latent_bench.log 2>&1 || { tail gpurun_out/r04g/latent_bench.log; exit 1; }
grep '^{' gpurun_out/r04g/latent_bench.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r04g/lprof -o run -- python3 -u tools/latent_bench.py 100 > gpurun_out/r04g/latent_prof.log 2>&1 || { tail gpurun_out/r04g/latent_prof.log; exit 1; }
python3 tools/rocpd_summary.py $(find gpurun_out/r04g/lprof -name "*.db" | head -1) | sed -n '/hot path/,$p' | head -6
bash tools/gpu.sh r04g tests smoke bench:"--gpus 1 --steps 3 --warmup 1 --no-cpu-baseline" || exit 1
