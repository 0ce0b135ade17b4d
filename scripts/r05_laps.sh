#!/bin/bash
# round 5: GPU suite, then stamped laps of the read/lower pipeline at pop 1M
# (C3) and C3/C5 end to end
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r05_laps_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05_laps_tests.log; [ $rc -eq 0 ] || exit $rc
GPE_DIAG=1 timeout -k 10 200 python3 -u scripts/e2e_phases.py c3 8 > gpurun_out/laps_c3.log 2>&1 || exit 1
grep -E "read_lower|metadata|^total" gpurun_out/laps_c3.log | tail -17
for rep in 1 2; do
  timeout -k 10 300 python3 scripts/bench_configs.py --only c3,c5 --reps 7 2>&1 | grep '^{' | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['config'], r['kernel_ms'], r['device_ms'], r['e2e_ms'], sorted(r['e2e_ms_all'])[3])" || exit 1
done
