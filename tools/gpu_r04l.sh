set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04l
timeout -k 10 300 python -u tools/layout_bench.py > gpurun_out/r04l/layout.log 2>&1 || { tail gpurun_out/r04l/layout.log; exit 1; }
grep '^{' gpurun_out/r04l/layout.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04l/lprof -o run -- python3 -u tools/layout_bench.py > gpurun_out/r04l/layout_prof.log 2>&1 || { tail gpurun_out/r04l/layout_prof.log; exit 1; }
python3 tools/rocpd_summary.py $(find gpurun_out/r04l/lprof -name "*.db" | head -1) | sed -n '/hot path/,$p' | head -6
