#!/bin/bash
# Round 6 same-box A/Bs, interleaved: where the exact sin/cos handlers drop to
# their low wave priority — after their table gathers land (default), as soon
# as they are issued (dissue), after the range blocks (djoin) — and sin/cos +
# protectedDiv at 1 instead of 0 / 1 (late1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/ab.sh "wait:X=1" "dissue:DEAP_AMD_LIB=deap_amd/libgpeval_dissue.so" \
  "djoin:DEAP_AMD_LIB=deap_amd/libgpeval_djoin.so" "late1:DEAP_AMD_LIB=deap_amd/libgpeval_late1.so" \
  "wait2:X=1" "dissue2:DEAP_AMD_LIB=deap_amd/libgpeval_dissue.so" \
  "djoin2:DEAP_AMD_LIB=deap_amd/libgpeval_djoin.so" "late12:DEAP_AMD_LIB=deap_amd/libgpeval_late1.so"
