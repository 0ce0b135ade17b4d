#!/bin/bash
# Per-shard (strong-scaling) prediction on one GPU: bench.py at the case
# counts one rank of N = 2, 4, 8 holds (2^20 / N), then configs 3 and 5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in 1048576 524288 262144 131072; do
  timeout -k 10 200 python -u bench.py --cases $c --no-cpu-baseline --no-fp32 --no-trig-leaves --steps 5 --warmup 2 > gpurun_out/shard_$c.log 2>&1
  rc=$?; echo "cases=$c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - gpurun_out/shard_$c.log <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
g = r["config"]["geometry"]
print("  value %.1f ms_per_step %.2f kernel_ms %.2f P %s groups %s redo %s"
      % (r["value"], r["ms_per_step"], r["roofline"]["kernel_ms"], g["P"], g["groups"], g["redo"]))
PY
done
timeout -k 10 400 python -u scripts/bench_configs.py --only c2,c3,c5 --reps 2 > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
rc=$?; echo "configs rc=$rc"; cat gpurun_out/configs.jsonl
