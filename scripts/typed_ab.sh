#!/bin/bash
# A/B of the typed core's block geometry on C5 (pop 1M): kernel ms per variant.
# Usage: bash scripts/typed_ab.sh "tag:ENV=val ..." ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}
  timeout -k 10 200 env $envs python3 -u scripts/bench_configs.py --only ${AB_CFG:-c5} --reps 3 \
      > gpurun_out/tab_$tag.jsonl 2>&1 || { echo "$tag failed"; tail -n 5 gpurun_out/tab_$tag.jsonl; exit 1; }
  python3 -c "
import json, sys
for l in open('gpurun_out/tab_$tag.jsonl'):
    if l.startswith('{'):
        d = json.loads(l)
        g = d['geometry']
        print('%-8s %s kernel_ms=%.3f gpops=%.0f device_ms=%.1f e2e_ms=%.1f P=%s groups=%s' % ('$tag', d['config'], d['kernel_ms'], d['kernel_gpops'], d['device_ms'], d['e2e_ms'], g.get('asm_typed_P'), g.get('asm_typed_groups')))
"
done
