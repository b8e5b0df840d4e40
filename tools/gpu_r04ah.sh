# refreshed PMC of the cross kernels after the round-4 work-order / prefetch changes
set -u
export TMPDIR=/tmp
for spec in "x80r4:tools/cross_one.py:20,edit+store,1024,80" "x160r4:tools/cross_one.py:20,edit+store,256,160" \
            "x40grpr4:tools/cross_one.py:20,edit,4096,40"; do
  bash tools/gpu.sh r04ah "pmcs:$spec" || exit 1
done
