#!/bin/bash
# Kernel trace + stats of one bench configuration (no PMC).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-quick}
out=gpurun_out/trace_$tag
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
  python3 bench.py --no-cpu-baseline --no-side-configs --no-trig-leaves --no-fp32 --steps 2 --warmup 1 > $out/bench.log 2>&1
rc=$?; echo "trace rc=$rc"
f=$(find $out -name "run_kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -d, -f1-4 "$f" | head -8
exit $rc
