#!/bin/bash
# Round 6 same-box A/B, interleaved: the exact launches' LDS budget priced
# with their own (glibc) table instead of the table core's, which admits a
# sixth program per wave on C4 (GPE_ASM_P=5: the old P); then the exact-core
# parity tests on the new geometry.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/ab.sh "p6:X=1" "p5:GPE_ASM_P=5" "p6b:X=1" "p5b:GPE_ASM_P=5" || exit $?
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -v -s --timeout 300 \
  --timeout-method thread -k "exact_asm_core_sin_cos or headline_workload or bench_hard or \
c4_symreg10 or deep_asm_core_matches or evolved_population or planner_state or \
headline_population_matches or abandoned" > gpurun_out/r06_t17.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|bit-identical|passed|failed" gpurun_out/r06_t17.log | tail -20
exit $rc
