#!/bin/bash
# round 5: GPU suite, then C2/C3/C5 end to end (bench_configs, 7 reps)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
  > gpurun_out/r05_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/r05_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python3 scripts/bench_configs.py --only c2,c3,c5 --reps 7 2>&1 | grep '^{' | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['config'], r['kernel_ms'], r['device_ms'], r['e2e_ms'], sorted(r['e2e_ms_all'])[3])" || exit 1
done
