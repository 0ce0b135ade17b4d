#!/bin/bash
# Round 6 same-box A/B, interleaved: larger planner weights (GPE_TRIG_W,
# GPE_DIV_W) around the best of scripts/r06_gpu13.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/ab.sh "t10d3:GPE_TRIG_W=10 GPE_DIV_W=3" "t12d4:GPE_TRIG_W=12 GPE_DIV_W=4" \
  "t14d5:GPE_TRIG_W=14 GPE_DIV_W=5" "t16d6:GPE_TRIG_W=16 GPE_DIV_W=6" \
  "t12d3:GPE_TRIG_W=12 GPE_DIV_W=3" \
  "t10d3b:GPE_TRIG_W=10 GPE_DIV_W=3" "t12d4b:GPE_TRIG_W=12 GPE_DIV_W=4" \
  "t14d5b:GPE_TRIG_W=14 GPE_DIV_W=5" "t16d6b:GPE_TRIG_W=16 GPE_DIV_W=6" \
  "t12d3b:GPE_TRIG_W=12 GPE_DIV_W=3"
