# round 4: tests for the changed paths, cross A/B, PMC of every attention kernel (verdict r03 item 2), bench
set -u
export TMPDIR=/tmp
bash tools/gpu.sh r04c files:tests/test_gpu_latent.py,tests/test_gpu_blend_fold.py \
  tests:"teacher_forced or cross_group_kernel or cross_edit_paths or edits_bf16_sd_geometry" || exit 1
CROSS_BENCH_GRAPH=1 timeout -k 10 300 python -u tools/cross_bench.py > gpurun_out/r04c/cross_bench.log 2>&1 || { tail -5 gpurun_out/r04c/cross_bench.log; exit 1; }
grep '^{' gpurun_out/r04c/cross_bench.log
for spec in "s80:tools/g1_only.py:20,1024,80" "s160ring:tools/g1_only.py:20,256,160" "s160split:tools/g1_only.py:20,64,160" \
            "x80:tools/cross_one.py:20,edit+store,1024,80" "x160:tools/cross_one.py:20,edit+store,256,160" \
            "x40grp:tools/cross_one.py:20,edit,4096,40"; do
  bash tools/gpu.sh r04c "pmcs:$spec" || exit 1
done
bash tools/gpu.sh r04c bench:"--gpus 1 --steps 3 --warmup 1 --no-cpu-baseline" || exit 1
