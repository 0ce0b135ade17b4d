#!/bin/bash
# round 5: the read+lower pipeline's laps at pop 1M (C3, C5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in c3 c5; do
  echo "== $c diag"
  GPE_DIAG=1 timeout -k 10 200 python3 -u scripts/e2e_phases.py $c 4 > gpurun_out/diag3_$c.log 2>&1 || exit 1
  grep -E "read_lower|gpe_lower_add|gpe_lower_end|run_common plan|^total" gpurun_out/diag3_$c.log | tail -24
done
