#!/bin/bash
# Round 6 pricing A/Bs on the final exact core (trig weight 8), interleaved:
# a third __sincostab gather per call and case (dup_tab) and six more SALU per
# sin/cos call (dup_salu); then the typed core's PMC passes (C5 at pop 1M).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/ab.sh "base:X=1" "duptab:DEAP_AMD_LIB=deap_amd/libgpeval_duptab.so" \
  "dupsalu:DEAP_AMD_LIB=deap_amd/libgpeval_dupsalu.so" \
  "baseb:X=1" "duptabb:DEAP_AMD_LIB=deap_amd/libgpeval_duptab.so" \
  "dupsalub:DEAP_AMD_LIB=deap_amd/libgpeval_dupsalu.so" || exit $?
bash scripts/r05_typed_pmc.sh
