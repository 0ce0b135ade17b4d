#!/bin/bash
# round 5: kernel + copy traces of evaluate at pop 1M (C3, C5), final build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in c3 c5; do
  rm -rf gpurun_out/prof_e2e_$c
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_e2e_$c -o $c -- python3 -u scripts/e2e_phases.py $c 5 > gpurun_out/prof_e2e_$c.log 2>&1 || exit 1
  grep "^total" gpurun_out/prof_e2e_$c.log
done
