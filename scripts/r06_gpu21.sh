#!/bin/bash
# Round 6 same-box A/B at six programs per wave, interleaved: the planner
# weights around (14, 5), one tile buffer (P = 7), the exact launch's grid
# target.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/ab.sh "base:X=1" "t10d4:GPE_TRIG_W=10 GPE_DIV_W=4" "t18d6:GPE_TRIG_W=18 GPE_DIV_W=6" \
  "nodbuf:GPE_ASM_DBUF=0" "xt32k:GPE_XASM_TARGET_BLOCKS=32768" "xt128k:GPE_XASM_TARGET_BLOCKS=131072" \
  "baseb:X=1" "t10d4b:GPE_TRIG_W=10 GPE_DIV_W=4" "t18d6b:GPE_TRIG_W=18 GPE_DIV_W=6" \
  "nodbufb:GPE_ASM_DBUF=0" "xt32kb:GPE_XASM_TARGET_BLOCKS=32768" "xt128kb:GPE_XASM_TARGET_BLOCKS=131072"
