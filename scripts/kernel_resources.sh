#!/bin/bash
# Registers, spills and LDS of the gfx950 kernels in libgpeval.so, read from
# the code object's metadata (the round-2 check that f_eval_asm does not
# spill).  Usage: scripts/kernel_resources.sh [filter-regex]
set -euo pipefail
LIB=${LIB:-$(dirname "$0")/../deap_amd/libgpeval.so}
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
objcopy --dump-section .hip_fatbin="$TMP/fatbin.bin" "$LIB" /dev/null
/opt/rocm/llvm/bin/clang-offload-bundler --unbundle --type=o \
  --input="$TMP/fatbin.bin" --output="$TMP/gfx950.co" \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950
/opt/rocm/llvm/bin/llvm-readelf --notes "$TMP/gfx950.co" > "$TMP/notes.txt"
python3 - "$TMP/notes.txt" "${1:-.}" <<'PY'
import re, sys
text = open(sys.argv[1]).read()
pat = re.compile(sys.argv[2])
for block in text.split("  - .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", block).group(1)
    if not pat.search(name):
        continue
    get = lambda k: (re.search(r"\.%s:\s+(\S+)" % k, block) or [None, "?"])[1]
    print("%-60s vgpr %3s spill %3s sgpr %3s sgpr_spill %3s lds %6s scratch %4s"
          % (name[:60], get("vgpr_count"), get("vgpr_spill_count"),
             get("sgpr_count"), get("sgpr_spill_count"),
             get("group_segment_fixed_size"),
             get("private_segment_fixed_size")))
PY
