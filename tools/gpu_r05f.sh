set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r05f
timeout -k 10 400 python -u -m pytest -x -v -s --durations=5 --timeout 300 --timeout-method thread -m gpu "tests/test_gpu_bench_config.py::test_config2_eight_refine_reweight_groups_vs_oracle" tests/test_gpu_bench_config.py::test_bench_config_sharpened_50_steps > gpurun_out/r05f/default.log 2>&1 || { tail -30 gpurun_out/r05f/default.log; exit 1; }
tail -12 gpurun_out/r05f/default.log
MIOPEN_FIND_MODE=FAST timeout -k 10 400 python -u -m pytest -x -v -s --durations=5 --timeout 300 --timeout-method thread -m gpu "tests/test_gpu_bench_config.py::test_config2_eight_refine_reweight_groups_vs_oracle" > gpurun_out/r05f/fast.log 2>&1 || { tail -30 gpurun_out/r05f/fast.log; exit 1; }
tail -8 gpurun_out/r05f/fast.log
