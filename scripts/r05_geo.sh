#!/bin/bash
# round 5: launch geometry of the exact core (programs per wave, grid target)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export AB_ARGS="--no-trig-leaves --no-fp32"
bash scripts/ab.sh "base:X=1" "p4:GPE_ASM_P=4" "p6:GPE_ASM_P=6" "p8:GPE_ASM_P=8" \
  "t32k:GPE_XASM_TARGET_BLOCKS=32768" "t128k:GPE_XASM_TARGET_BLOCKS=131072" "base2:X=2"
