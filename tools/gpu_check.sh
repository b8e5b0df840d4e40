set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== attn bench"; timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1; rc=$?; cat gpurun_out/attn_bench.log | grep -E "geom|variant"; echo "rc=$rc"
exit $rc
