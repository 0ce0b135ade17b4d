#!/bin/bash
# round 5: C3 / C5 evaluate end to end (bench_configs, best of reps), phases
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python3 -u scripts/bench_configs.py --only c3,c5,c5_real --reps 7 \
    > gpurun_out/r05_e2e_$r.log 2>&1 || exit 1
  grep "^{" gpurun_out/r05_e2e_$r.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(' ', r.get('config'), 'e2e_ms', r.get('e2e_ms'), 'device_ms', r.get('device_ms'), 'kernel_ms', r.get('kernel_ms'))"
done
for c in c3 c5; do
  echo "== $c"; timeout -k 10 200 python3 -u scripts/e2e_phases.py $c 21 2>&1 | grep -v amdgpu.ids || exit 1
done
