#!/bin/bash
# Host phases of evaluate at pop 1M (C3, C5): native laps (GPE_DIAG) and a
# cProfile of one warm call.  Usage: r04_e2e.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-r04}
for c in c3 c5; do
  timeout -k 10 240 env GPE_DIAG=1 python3 -u scripts/e2e_profile.py $c 30 \
    > gpurun_out/${tag}_e2e_$c.log 2>&1 || exit 1
  grep "evaluate" gpurun_out/${tag}_e2e_$c.log | head -3
done
