#!/bin/bash
# Generic GPU step runner: each step under its own time limit; stop at the first failure.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  grep -v "amdgpu.ids" gpurun_out/$name.log | tail -${TAIL:-15}
  echo "rc=$rc"
  return $rc
}
