#!/bin/bash
# One gpurun call WITH the experiments library (p2p_amd/exp/libp2p_hip.so, built here first) in the
# push: .gpurunignore keeps it out of every other call (tests, smoke and bench never load it); this
# wrapper drops that line for this call only and restores the file afterwards.
#   tools/gpu_ab.sh --timeout 600 -- 'bash tools/gpu.sh <tag> stamps:cross_stamps:90 ...'
set -u
cd "$(dirname "$0")/.."
make -C prompt-to-prompt_amd/csrc EXPERIMENTS=1 -j8 > /tmp/make_exp.log 2>&1 || { tail -20 /tmp/make_exp.log; exit 1; }
bak=$(mktemp /tmp/gpurunignore.XXXXXX)
cp .gpurunignore "$bak"
# restore the tracked file however this script ends (error, Ctrl-C, kill)
trap 'cp "$bak" .gpurunignore; rm -f "$bak"' EXIT
trap 'exit 130' INT TERM
grep -v '^\./prompt-to-prompt_amd/p2p_amd/exp$' "$bak" > .gpurunignore
/usr/local/graft/bin/gpurun "$@"
