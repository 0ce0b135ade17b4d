#!/bin/bash
# round 5: evaluate phases at pop 1M (C3, C5), the native read+lower pipeline on / off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in c3 c5; do
  for v in 1 0 1 0; do
    echo "== $c read_lower=$v"
    GPE_READ_LOWER=$v timeout -k 10 200 python3 -u scripts/e2e_phases.py $c 21 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
