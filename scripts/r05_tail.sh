#!/bin/bash
# round 5: evaluate at pop 1M (C3, C5) by the lowering's tail chunks
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in c3 c5; do
  for rep in 1 2 3; do
    for tail in 16384 65536 0; do
      echo "== $c tail=$tail"
      GPE_LOWER_TAIL=$tail timeout -k 10 200 python3 -u scripts/e2e_phases.py $c 21 2>&1 | grep -E "^total" || exit 1
    done
  done
done
