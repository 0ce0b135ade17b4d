#!/bin/bash
# Per-shard strong-scaling prediction on one GPU (bench.py at the case count
# one rank of N = 1/2/4/8 holds) and a kernel trace of the world-1 sharded
# path at 2^17 cases (RCCL redo-flag all-reduce, device compaction of the
# redo list): the gaps between the main kernel and the redo pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r04}
out=gpurun_out/shard_$tag
mkdir -p $out
: > $out/scaling.jsonl
for c in 1048576 524288 262144 131072; do
  timeout -k 10 200 python3 -u bench.py --cases $c --steps 5 --warmup 2 --no-cpu-baseline \
    --no-side-configs --no-trig-leaves --no-fp32 > $out/n_$c.log 2>&1 || exit 1
  grep "^{" $out/n_$c.log >> $out/scaling.jsonl
done
python3 - $out/scaling.jsonl <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
t1 = rows[0]["ms_per_step"]
for r, n in zip(rows, (1, 2, 4, 8)):
    print(r["config"]["cases"], r["ms_per_step"], round(t1 / n, 2), round(t1 / n / r["ms_per_step"], 3))
PY
DEAP_AMD_FORCE_DIST=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29519 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 \
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- \
  python3 bench.py --cases 131072 --steps 3 --warmup 1 --no-cpu-baseline --no-side-configs \
  --no-trig-leaves --no-fp32 > $out/dist1_trace.log 2>&1
rc=$?; echo "dist trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $out/trace -name "run_kernel_trace.csv" | head -1)
python3 scripts/kernel_gaps.py "$f" 10 > $out/gaps.txt
tail -25 $out/gaps.txt | cut -c1-200
