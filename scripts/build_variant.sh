#!/bin/bash
# Build an experimental variant of libgpeval.so (for DEAP_AMD_LIB A/B runs):
#   scripts/build_variant.sh <name> [ENV=val ...]   -> deap_amd/libgpeval_<name>.so
# The generator environment (e.g. GEN_ASM_EXPERIMENT=..., GEN_ASM_TRIG_GROUP=2)
# applies to the regenerated fp64 asm cores.  ASM_K / ASM_DEEP_K / ASM_EXACT_K /
# ASM_NV: cases per lane and variables of the cores.  The variant is generated
# and compiled in a scratch copy of the sources, so several builds may run at
# once and the tree's own generated cores are never touched.
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; shift
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
mkdir -p "$tmp/deap_amd/csrc" "$tmp/include"
cp include/gpeval.h "$tmp/include/"
cp deap_amd/csrc/gpeval.hip deap_amd/csrc/lower_core.h deap_amd/csrc/host_pool.h deap_amd/csrc/bigint_host.h \
   deap_amd/csrc/trig_dev.h deap_amd/csrc/exact_int.h deap_amd/csrc/rccl_layer.h deap_amd/csrc/select_dev.h \
   deap_amd/csrc/ctx.h deap_amd/csrc/fb_kernels.h deap_amd/csrc/asm_kernels.h \
   deap_amd/csrc/planner.h deap_amd/csrc/exact_run.h \
   deap_amd/csrc/gp_asm_core32*.inc \
   "$tmp/deap_amd/csrc/"
K=${ASM_K:-2}
NV=${ASM_NV:-32}
out="$tmp/deap_amd/csrc"
for kv in "$@"; do export "$kv"; done
gen() { python3 -c "
import sys; sys.path.insert(0, 'deap_amd/csrc'); import gen_asm
a = sys.argv[1:6] + ["0"]
gen_asm.emit(int(a[0]), int(a[1]), int(a[2]), a[3], out_dir='$out', trig_group=int(a[4]))" "$@"; }
gen $K ${ASM_D:-5} $NV "" ${ASM_TG:-0}
gen ${ASM_DEEP_K:-2} 12 $NV _deep
gen ${ASM_EXACT_K:-2} 5 $NV _exact
gen 2 5 64 _typed
gen ${ASM_EXACT_K:-2} 12 $NV _exact_deep
# the fp32 cores too (GEN_ASM32_* switches) when ASM32_REGEN=1
if [ "${ASM32_REGEN:-0}" = 1 ]; then
  for a in "4 5 32 ''" "4 12 32 _deep"; do
    eval "set -- $a"
    python3 -c "
import sys; sys.path.insert(0, 'deap_amd/csrc'); import gen_asm32
gen_asm32.emit(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], out_dir='$out')" "$@"
  done
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared -std=c++17 \
  -Wno-unused-function ${HIPFLAGS:-} "$out/gpeval.hip" -o deap_amd/libgpeval_$name.so
echo "built deap_amd/libgpeval_$name.so"
