#!/bin/bash
# Round-2 GPU call: headline parity test, counter list, profile passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -v --timeout 250 --timeout-method thread -k "headline or trig or rccl or c_abi or sharded" > gpurun_out/gpu_headline.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/gpu_headline.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1
echo "list rc=$?"
BENCH_ARGS="--no-cpu-baseline --no-trig-leaves --no-fp32 --steps 2 --warmup 1" bash scripts/profile.sh r02a
