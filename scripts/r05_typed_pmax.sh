#!/bin/bash
# round 5: typed core programs per wave (C5 at pop 1M): the wave's code windows
# are re-read from the scalar cache every tile (64 programs x ~6 words per wave)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for p in 64 32 16 8; do
    echo "== pmax $p: $(GPE_TYPED_PMAX=$p timeout -k 10 200 python3 scripts/bench_configs.py --only c5 --reps 5 2>&1 | grep '^{' | python3 -c "
import json,sys; r=json.loads(sys.stdin.read()); print(r['kernel_ms'], r['e2e_ms'], r['geometry'].get('asm_typed_P'), r['geometry'].get('asm_typed_groups'))")"
  done
done
