#!/bin/bash
# round 5: evaluate phases at pop 1M (C3, C5) with gpe_lower_end's laps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in c3 c5; do
  echo "== $c"
  timeout -k 10 200 python3 -u scripts/e2e_phases.py $c 21 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== $c diag"
  GPE_DIAG=1 timeout -k 10 200 python3 -u scripts/e2e_phases.py $c 3 > gpurun_out/diag_$c.log 2>&1 || exit 1
  grep -E "gpe_lower_end|plan|run_common" gpurun_out/diag_$c.log | tail -30
done
