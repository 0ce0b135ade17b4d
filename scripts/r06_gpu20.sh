#!/bin/bash
# Round 6: the exact core's dynamic program order (the block's waves take
# their programs from an LDS counter per tile; GPE_DYN=0: each wave its own
# list) — the exact-core parity tests on it first, then a same-box A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -v -s --timeout 300 \
  --timeout-method thread -k "exact_asm_core_sin_cos or headline_workload or bench_hard or \
c4_symreg10 or deep_asm_core_matches or evolved_population or planner_state or \
headline_population_matches or abandoned or c1_ or exact_int" > gpurun_out/r06_t20.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|bit-identical|passed|failed" gpurun_out/r06_t20.log | tail -30
[ $rc -eq 0 ] || exit $rc
bash scripts/ab.sh "dyn:X=1" "static:GPE_DYN=0" "dynb:X=1" "staticb:GPE_DYN=0"
