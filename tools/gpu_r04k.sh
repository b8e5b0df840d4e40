set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04k
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r04k/cprof -o run -- python3 -u tools/clock_check.py 50 > gpurun_out/r04k/clock.log 2>&1 || { tail gpurun_out/r04k/clock.log; exit 1; }
grep '^{' gpurun_out/r04k/clock.log
python3 tools/rocpd_summary.py $(find gpurun_out/r04k/cprof -name "*.db" | head -1) | sed -n '/hot path/,$p' | head -6
bash tools/gpu.sh r04k ab:0,165,0,165 stamps:s40_stamps:163 stamps:s40_stamps:166 || exit 1
