#!/bin/bash
# round 5: C3 / C5 evaluate end to end, tail chunks on / off (same box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 1 0 1 0; do
  GPE_LOWER_TAIL=$v timeout -k 10 300 python3 -u scripts/bench_configs.py --only c3,c5 --reps 7 \
    > gpurun_out/r05_e2e_tail$v.log 2>&1 || exit 1
  echo "tail=$v"; grep "^{" gpurun_out/r05_e2e_tail$v.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(' ', r.get('config'), 'e2e_ms', r.get('e2e_ms'), 'device_ms', r.get('device_ms'), 'kernel_ms', r.get('kernel_ms'))"
done
