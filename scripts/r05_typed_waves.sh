#!/bin/bash
# round 5: typed core waves per block (C5 at pop 1M): 8 (4 waves/SIMD: LDS) vs
# 10 (5 waves/SIMD: two 59 KB blocks per CU, 82 VGPRs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for w in 8 10 6; do
    echo "== waves $w: $(GPE_TYPED_WAVES=$w timeout -k 10 200 python3 scripts/bench_configs.py --only c5 --reps 5 2>&1 | grep '^{' | python3 -c "
import json,sys; r=json.loads(sys.stdin.read()); print(r['kernel_ms'], r['e2e_ms'], r['geometry'].get('asm_typed_P'), r['geometry'].get('asm_typed_groups'))")"
  done
done
