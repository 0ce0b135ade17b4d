#!/bin/bash
# round 5: split evaluate — GPU suite, then evaluate at pop 1M (C3, C5), split on / off
# (historical: split evaluation and its GPE_SPLIT_MIN knob were dropped)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r05_split_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05_split_tests.log; [ $rc -eq 0 ] || exit $rc
for c in c3 c5; do
  for rep in 1 2; do
    for sm in 524288 0; do
      echo "== $c split_min=$sm"
      GPE_SPLIT_MIN=$sm timeout -k 10 200 python3 -u scripts/e2e_phases.py $c 21 2>&1 | grep -E "^total" || exit 1
    done
  done
done
