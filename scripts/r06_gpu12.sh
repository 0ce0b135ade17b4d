#!/bin/bash
# Round 6 same-box A/B, interleaved: the planner's protectedDiv weight
# (GPE_DIV_W: code words per protectedDiv node added to a program's cost).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/ab.sh "d0:X=1" "d2:GPE_DIV_W=2" "d4:GPE_DIV_W=4" "d8:GPE_DIV_W=8" \
  "d0b:X=1" "d2b:GPE_DIV_W=2" "d4b:GPE_DIV_W=4" "d8b:GPE_DIV_W=8"
