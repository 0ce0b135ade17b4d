#!/bin/bash
# round 5: lowering on two streams — tests, phases at pop 1M (tail halving on/off), C3 trace
# (historical: GPE_LOWER_TAIL now takes a chunk size >= 1024; 0/1 both mean no tail)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r05_lw3_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05_lw3_tests.log; [ $rc -eq 0 ] || exit $rc
for c in c3 c5; do
  for tail in 1 0 1 0; do
    echo "== $c tail=$tail"
    GPE_LOWER_TAIL=$tail timeout -k 10 200 python3 -u scripts/e2e_phases.py $c 21 2>&1 | grep -E "total|lower_end|run " || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_c3b -o c3 -- python3 -u scripts/e2e_phases.py c3 5 > gpurun_out/prof_c3b.log 2>&1 || exit 1
echo prof ok
