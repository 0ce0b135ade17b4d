#!/bin/bash
# Round 6 same-box A/Bs on the glibc_seq4 exact core, interleaved:
# new (the default: M0 in a VGPR lane, the range compares early) vs noearly
# (GEN_ASM_EARLY=0); and the wave-priority schemes on the noearly build:
# tiered_late (noearly itself), none (pnone), tiered (ptier: sin/cos at 0 from
# entry), trig_low (plow: two levels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/ab.sh "new:X=1" "noearly:DEAP_AMD_LIB=deap_amd/libgpeval_noearly.so" \
  "pnone:DEAP_AMD_LIB=deap_amd/libgpeval_pnone.so" "ptier:DEAP_AMD_LIB=deap_amd/libgpeval_ptier.so" \
  "plow:DEAP_AMD_LIB=deap_amd/libgpeval_plow.so" \
  "new2:X=1" "noearly2:DEAP_AMD_LIB=deap_amd/libgpeval_noearly.so" \
  "pnone2:DEAP_AMD_LIB=deap_amd/libgpeval_pnone.so" "ptier2:DEAP_AMD_LIB=deap_amd/libgpeval_ptier.so" \
  "plow2:DEAP_AMD_LIB=deap_amd/libgpeval_plow.so"
