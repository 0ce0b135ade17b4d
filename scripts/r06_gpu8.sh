#!/bin/bash
# Round 6 same-box A/B, interleaved: the planner's sin/cos weight in the
# program cost that deals programs to waves (GPE_TRIG_W; default 14), and
# the order of a wave's programs (GPE_DEAL_MIX: 1 odd waves reversed, 2 wave
# wv starts at band wv mod P).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/ab.sh "w14:X=1" "w8:GPE_TRIG_W=8" "w4:GPE_TRIG_W=4" "w0:GPE_TRIG_W=0" \
  "w8m1:GPE_TRIG_W=8 GPE_DEAL_MIX=1" "w8m2:GPE_TRIG_W=8 GPE_DEAL_MIX=2" \
  "w14b:X=1" "w8b:GPE_TRIG_W=8" "w4b:GPE_TRIG_W=4" "w0b:GPE_TRIG_W=0" \
  "w8m1b:GPE_TRIG_W=8 GPE_DEAL_MIX=1" "w8m2b:GPE_TRIG_W=8 GPE_DEAL_MIX=2"
