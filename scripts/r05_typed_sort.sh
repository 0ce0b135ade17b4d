#!/bin/bash
# round 5: the typed launch's plan with / without the cost sort (C5 at pop 1M)
# (the GPE_TYPED_SORT knob this A/B used is gone: large typed launches skip the sort)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2 3; do
  for t in 1 0; do
    echo "== sort=$t: $(GPE_TYPED_SORT=$t timeout -k 10 200 python3 scripts/bench_configs.py --only c5 --reps 7 2>&1 | grep '^{' | python3 -c "
import json,sys; r=json.loads(sys.stdin.read()); print(r['kernel_ms'], r['device_ms'], r['e2e_ms'], sorted(r['e2e_ms_all'])[3])")"
  done
done
