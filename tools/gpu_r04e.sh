set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04e
bash tools/gpu.sh r04e files:tests/test_gpu_latent.py,tests/test_gpu_blend_fold.py tests:"cross_group_kernel or cross_edit_paths or edits_bf16_sd_geometry" || exit 1
timeout -k 10 120 python -u tools/latent_bench.py > gpurun_out/r04e/latent_bench.log 2>&1 || { tail gpurun_out/r04e/latent_bench.log; exit 1; }
grep '^{' gpurun_out/r04e/latent_bench.log
CROSS_BENCH_GRAPH=1 timeout -k 10 300 python -u tools/cross_bench.py > gpurun_out/r04e/cross_bench.log 2>&1 || { tail -5 gpurun_out/r04e/cross_bench.log; exit 1; }
grep '^{' gpurun_out/r04e/cross_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04e/prof -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r04e/prof.log 2>&1 || { tail gpurun_out/r04e/prof.log; exit 1; }
python3 tools/rocpd_summary.py $(find gpurun_out/r04e/prof -name "*.db" | head -1) > gpurun_out/r04e/rocprof_summary.txt; sed -n '/hot path/,$p' gpurun_out/r04e/rocprof_summary.txt | head -16
