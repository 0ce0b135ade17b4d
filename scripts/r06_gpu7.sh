#!/bin/bash
# Round 6 same-box A/B, interleaved: END prefetches the next program's first
# code window (GEN_ASM_PF=1, libgpeval_pf.so) against the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/ab.sh "base:X=1" "pf:DEAP_AMD_LIB=deap_amd/libgpeval_pf.so" \
  "base2:X=1" "pf2:DEAP_AMD_LIB=deap_amd/libgpeval_pf.so" \
  "base3:X=1" "pf3:DEAP_AMD_LIB=deap_amd/libgpeval_pf.so"
