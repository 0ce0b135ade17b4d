#!/bin/bash
# Round 6: (1) the C4 parity tests on a deliberately wrong core
# (libgpeval_ulp1.so: one ulp off on ~1/1024 of the exact sin/cos results;
# they must fail), (2) same-box A/Bs: protectedDiv's quotient into T with
# one select (default) vs the temporary + two selects (divold); the rare
# sin/cos blocks out of line (default) vs in line (inl); 40 extra lane ops
# per wave-tile (GPE_DIAG=16: the price of the SGPR spills' lane ops).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DEAP_AMD_LIB=deap_amd/libgpeval_ulp1.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py \
  -v --timeout 240 --timeout-method thread -k "headline_workload or bench_hard or \
exact_asm_core_sin_cos or headline_population_matches" \
  > gpurun_out/r06_ulp1.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r06_ulp1.log | tail -8
[ $rc -le 1 ] || exit $rc
bash scripts/ab.sh "divold:DEAP_AMD_LIB=deap_amd/libgpeval_divold.so" "new:X=1" \
  "inl:DEAP_AMD_LIB=deap_amd/libgpeval_inl.so" "spill40:GPE_DIAG=16" \
  "divold2:DEAP_AMD_LIB=deap_amd/libgpeval_divold.so" "new2:X=1" \
  "inl2:DEAP_AMD_LIB=deap_amd/libgpeval_inl.so" "spill40b:GPE_DIAG=16"
