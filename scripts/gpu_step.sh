#!/bin/bash
# One GPU-box session during development: the GPU suite, then the
# per-config throughput of the given configs and a short headline bench.
# Stops at the first step that fails.  Usage: bash scripts/gpu_step.sh <tag> [configs]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-dev}
cfgs=${2:-c2,c3,c5}
timeout -k 10 400 python -u -m pytest tests/ -m gpu -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/${tag}_tests.log | head -20; tail -n 1 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_configs.py --only $cfgs --reps 3 > gpurun_out/${tag}_configs.jsonl 2> gpurun_out/${tag}_configs.err
rc=$?; echo "configs rc=$rc"; cut -c1-330 gpurun_out/${tag}_configs.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32 --steps 3 > gpurun_out/${tag}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep "^{" gpurun_out/${tag}_bench.log | cut -c1-250
exit $rc
