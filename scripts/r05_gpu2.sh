#!/bin/bash
# round 5: GPU suite, exact vs table A/B, a world-1 sharded bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -m gpu -v --timeout 200 \
    --timeout-method thread > gpurun_out/r05_t1.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r05_t1.log | tail -n 30
[ $rc -le 1 ] || exit $rc
bash scripts/ab.sh "exact:" "table:GPE_EXACT_ALL=0" || exit 1
MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 \
  DEAP_AMD_FORCE_DIST=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 \
  --no-cpu-baseline --no-side-configs --no-fp32 --no-trig-leaves > gpurun_out/r05_dist1.log 2>&1
echo "dist1 rc=$?"; grep "^{" gpurun_out/r05_dist1.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['value'], r.get('multi_gpu'))"
