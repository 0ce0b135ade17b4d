#!/bin/bash
# round 5: split evaluate laps at pop 1M (C5, C3)
# (historical: split evaluation was dropped)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in c5 c3; do
  echo "== $c"
  GPE_DIAG=1 timeout -k 10 200 python3 -u scripts/e2e_phases.py $c 3 > gpurun_out/split_$c.log 2>&1 || exit 1
  grep -E "^split|read_lower|gpe_run run|run_common plan|plan_mode|gpe_lower_end done|^total" gpurun_out/split_$c.log | tail -32
done
