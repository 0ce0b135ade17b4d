#!/bin/bash
# round 5: the typed-core parity test at 200K programs (program-order plan)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "typed_core_matches_cpp" > gpurun_out/typed_test.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/typed_test.log | tail -5; exit $rc
