#!/bin/bash
# Round 6: the typed core's END with its lane reads ahead of their users (no
# wait-state nops) — the C5 parity tests, the C5 kernel time (bench_configs),
# then the typed core's PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "c5 or typed or spambase" > gpurun_out/r06_t22.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r06_t22.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/bench_configs.py --only c5,c5_real --reps 3 > gpurun_out/r06_c5.log 2>&1 || exit $?
tail -n 4 gpurun_out/r06_c5.log
bash scripts/r05_typed_pmc.sh
