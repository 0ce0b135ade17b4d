#!/bin/bash
# round 5: smoke(), and the exact core at the case counts one rank of N = 2/4/8 holds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r05_smoke.log
for c in 1048576 524288 262144 131072; do
  timeout -k 10 300 python3 -u bench.py --cases $c --steps 3 --warmup 1 --no-cpu-baseline \
    --no-side-configs --no-fp32 --no-trig-leaves > gpurun_out/r05_shard_$c.log 2>&1 || exit 1
  grep "^{" gpurun_out/r05_shard_$c.log | python3 -c "
import json,sys; r=json.loads(sys.stdin.readline())
print(json.dumps({'cases': $c, 'ms_per_step': r['ms_per_step'], 'value': r['value'], 'kernel_ms': r['roofline']['kernel_ms']}))"
done | tee gpurun_out/r05_shard_scaling.jsonl
