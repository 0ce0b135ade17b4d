#!/bin/bash
# Round 2: cheaper sin/cos dispatch (16k rounding, operand constants) —
# parity subset, then same-box A/B against the previous library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "trig or headline or c4_ or random_shapes or deep_asm or c1_ or glibc or fp32_asm" > gpurun_out/r02_gpu6_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/r02_gpu6_tests.log
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--no-fp32 --no-trig-leaves --warmup 1" bash scripts/ab.sh "old:DEAP_AMD_LIB=deap_amd/libgpeval_old.so" "new:X=1" "old2:DEAP_AMD_LIB=deap_amd/libgpeval_old.so" "new2:X=2"
