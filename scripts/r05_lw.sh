#!/bin/bash
# round 5: lowering tests, then the evaluate phases at pop 1M (C3, C5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r05_lw_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05_lw_tests.log; [ $rc -eq 0 ] || exit $rc
for c in c3 c5; do
  echo "== $c"
  timeout -k 10 200 python3 -u scripts/e2e_phases.py $c 21 2>&1 | grep -v amdgpu.ids || exit 1
  GPE_DIAG=1 timeout -k 10 200 python3 -u scripts/e2e_phases.py $c 3 > gpurun_out/diag4_$c.log 2>&1 || exit 1
  grep -E "read_lower|gpe_lower_end|run_common plan" gpurun_out/diag4_$c.log | tail -10
done
