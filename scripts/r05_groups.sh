#!/bin/bash
# round 5: tiles per group at small case counts (a rank of N = 4/8), A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in 131072 262144 1048576; do
  for v in 128 0 128 0; do
    GPE_MIN_GROUP_TILES=$v timeout -k 10 300 python3 -u bench.py --cases $c --steps 3 --warmup 1 \
      --no-cpu-baseline --no-side-configs --no-fp32 --no-trig-leaves > gpurun_out/r05_grp_${c}_$v.log 2>&1 || exit 1
    grep "^{" gpurun_out/r05_grp_${c}_$v.log | python3 -c "
import json,sys; r=json.loads(sys.stdin.readline())
print($c, 'min_tiles', $v, 'ms', r['ms_per_step'], 'geo', r['config']['geometry']['groups'], r['config']['geometry']['P'])"
  done
done
