#!/bin/bash
# round 5: C3 at pop 1M, the lane-packed B kernel's plan with / without the cost sort
# (the GPE_B_SORT knob this A/B used is gone: program order became the default)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2 3; do
  for b in 1 0; do
    echo "== sort=$b: $(GPE_B_SORT=$b timeout -k 10 200 python3 scripts/bench_configs.py --only c3 --reps 7 2>&1 | grep '^{' | python3 -c "
import json,sys; r=json.loads(sys.stdin.read()); print(r['kernel_ms'], r['device_ms'], r['e2e_ms'], sorted(r['e2e_ms_all'])[3])")"
  done
done
