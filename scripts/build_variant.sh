#!/bin/bash
# Build an experimental variant of libgpeval.so (for DEAP_AMD_LIB A/B runs):
#   scripts/build_variant.sh <name> [ENV=val ...]   -> deap_amd/libgpeval_<name>.so
# The generator environment (e.g. GEN_ASM_EXPERIMENT=...) applies to the
# regenerated asm cores, which are restored afterwards.  ASM_K=1: one case
# per lane.
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; shift
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
cp deap_amd/csrc/gp_asm_core*.inc deap_amd/csrc/gp_asm_layout*.h "$tmp/"
K=${ASM_K:-2}
env "$@" python3 deap_amd/csrc/gen_asm.py $K 5 32 > /dev/null
env "$@" python3 deap_amd/csrc/gen_asm.py $K 12 32 _deep > /dev/null
env "$@" python3 deap_amd/csrc/gen_asm.py $K 5 32 _exact > /dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared -std=c++17 \
  -Wno-unused-function ${HIPFLAGS:-} deap_amd/csrc/gpeval.hip -o deap_amd/libgpeval_$name.so
cp "$tmp"/* deap_amd/csrc/
touch deap_amd/libgpeval.so
echo "built deap_amd/libgpeval_$name.so"
