#!/bin/bash
# round 5: GPU suite on the exact-core default, then A/B against the table cores
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -m gpu -v --timeout 200 \
    --timeout-method thread > gpurun_out/r05_t1.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r05_t1.log | tail -n 30
[ $rc -le 1 ] || exit $rc
bash scripts/ab.sh "exact:" "table:GPE_EXACT_ALL=0"
