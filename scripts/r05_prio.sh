#!/bin/bash
# round 5: wave priorities in the exact core (same-box A/B of variant builds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export AB_ARGS="--no-trig-leaves --no-fp32"
bash scripts/ab.sh "base:X=1" "pnone:DEAP_AMD_LIB=deap_amd/libgpeval_pnone.so" \
  "ptier:DEAP_AMD_LIB=deap_amd/libgpeval_ptier.so" "base2:X=2" \
  "pnone2:DEAP_AMD_LIB=deap_amd/libgpeval_pnone.so" "ptier2:DEAP_AMD_LIB=deap_amd/libgpeval_ptier.so"
