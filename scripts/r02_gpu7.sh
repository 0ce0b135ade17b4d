#!/bin/bash
# exact-redo trig over K cases at once: headline parity + trace; host CPU scaling probe
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "headline or glibc or random_shapes" > gpurun_out/r02_gpu7_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/r02_gpu7_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/trace_quick.sh k2exact || exit 1
gcc -O1 -pthread scripts/cpu_spin.c -o /tmp/cpu_spin && for t in 1 4 8 16; do /tmp/cpu_spin $t; done
