#!/bin/bash
# Round 6: the exact handlers with fewer SALU (GEN_ASM_SALU: EXEC saved once
# per core entry, v_cmpx for TAYLOR_SIN's lanes, the rare no-do_sin and
# reduce_sincos paths out of line) — the exact-core parity tests first, then
# a same-box A/B against GEN_ASM_SALU=0 (libgpeval_nosalu.so), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -v -s --timeout 300 \
  --timeout-method thread -k "exact_asm_core_sin_cos or device_glibc or \
headline_workload or bench_hard or c4_symreg10 or deep_asm_core_matches or \
evolved_population or planner_state or headline_population_matches" \
  > gpurun_out/r06_t10.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|bit-identical|passed|failed" gpurun_out/r06_t10.log | tail -30
[ $rc -eq 0 ] || exit $rc
bash scripts/ab.sh "salu:X=1" "nosalu:DEAP_AMD_LIB=deap_amd/libgpeval_nosalu.so" \
  "salub:X=1" "nosalub:DEAP_AMD_LIB=deap_amd/libgpeval_nosalu.so"
