#!/bin/bash
# Round 6: instruction-cache counters of the exact core (one PMC pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/prof_icache
rm -rf $out
timeout -s KILL 150 rocprofv3 --output-format csv --pmc SQC_ICACHE_REQ SQC_ICACHE_MISSES -d $out -o run -- python3 bench.py --no-cpu-baseline --no-side-configs --no-trig-leaves --no-fp32 --steps 1 --warmup 0 > $out.log 2>&1
rc=$?; echo "rc=$rc"; tail -n 3 $out.log; exit $rc
