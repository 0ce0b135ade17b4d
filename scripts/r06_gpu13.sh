#!/bin/bash
# Round 6 same-box A/B, interleaved: the planner's sin/cos and protectedDiv
# weights together (GPE_TRIG_W, GPE_DIV_W).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/ab.sh "t8d3:GPE_DIV_W=3" "t10d3:GPE_TRIG_W=10 GPE_DIV_W=3" \
  "t12d4:GPE_TRIG_W=12 GPE_DIV_W=4" "t6d2:GPE_TRIG_W=6 GPE_DIV_W=2" \
  "t8d3b:GPE_DIV_W=3" "t10d3b:GPE_TRIG_W=10 GPE_DIV_W=3" \
  "t12d4b:GPE_TRIG_W=12 GPE_DIV_W=4" "t6d2b:GPE_TRIG_W=6 GPE_DIV_W=2"
