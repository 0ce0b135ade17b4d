#!/bin/bash
# full GPU suite, then kernel trace of the headline and the C3/C5 e2e breakdown
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -v --timeout 200 --timeout-method thread \
  > gpurun_out/r02_gpu9_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r02_gpu9_tests.log | grep -v PASSED | head -20; tail -3 gpurun_out/r02_gpu9_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/trace_quick.sh r02b || exit 1
for cfg in c3 c5; do
  timeout -k 10 300 python -u scripts/e2e_breakdown.py $cfg > gpurun_out/host_${cfg}.log 2>&1 || exit 1
  grep "^{" gpurun_out/host_${cfg}.log
done
