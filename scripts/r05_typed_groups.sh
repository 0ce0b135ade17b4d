#!/bin/bash
# round 5: the typed launch's grid (C5 at pop 1M): target blocks -> tile groups
# (run with GPE_ASM_TARGET_BLOCKS before the typed launch had its own knob)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for tb in 65536 32768 131072 16384; do
    echo "== target $tb: $(GPE_TYPED_TARGET_BLOCKS=$tb timeout -k 10 200 python3 scripts/bench_configs.py --only c5 --reps 5 2>&1 | grep '^{' | python3 -c "
import json,sys; r=json.loads(sys.stdin.read()); print(r['kernel_ms'], r['e2e_ms'], r['geometry'].get('asm_typed_P'), r['geometry'].get('asm_typed_groups'))")"
  done
done
