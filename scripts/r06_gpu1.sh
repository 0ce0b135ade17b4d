#!/bin/bash
# Round 6, first GPU check of glibc_seq4 (the default build): the exact-core
# parity tests and the new reference-fixture tests, then a same-box A/B
# against glibc_seq3 (libgpeval_seq3.so, scripts/build_variant.sh seq3
# GEN_ASM_GLIBC4=0), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -v -s --timeout 300 \
  --timeout-method thread -k "exact_asm_core_sin_cos or device_glibc or \
headline_workload or bench_hard or c4_symreg10 or deep_asm_core_matches or \
evolved_population or c1_symbreg_golden or c1_edge or planner_state or \
headline_population_matches or evolved_population_matches_reference" \
  > gpurun_out/r06_t1.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|bit-identical|passed|failed" gpurun_out/r06_t1.log | tail -30
[ $rc -le 1 ] || exit $rc
bash scripts/ab.sh "seq3:DEAP_AMD_LIB=deap_amd/libgpeval_seq3.so" "seq4:X=1" \
  "seq3b:DEAP_AMD_LIB=deap_amd/libgpeval_seq3.so" "seq4b:X=1"
