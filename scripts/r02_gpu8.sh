#!/bin/bash
# exact asm core for the redo pass: trig bit-identity, parity, trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "exact_asm or headline or glibc or random_shapes or c4_ or trig" > gpurun_out/r02_gpu8_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/r02_gpu8_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/trace_quick.sh xasm
