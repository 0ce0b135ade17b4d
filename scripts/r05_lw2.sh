#!/bin/bash
# round 5: evaluate at pop 1M (C3, C5) by decode threads inside gpe_lower_add
# (historical: the GPE_LW_DEC_THREADS knob it varied is gone; the decode uses all host threads)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "lower or chunk" \
  > gpurun_out/r05_lw2_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05_lw2_tests.log; [ $rc -eq 0 ] || exit $rc
for c in c3 c5; do
  for t in 4 16 1 4 16 1; do
    echo "== $c dec_threads=$t"
    GPE_LW_DEC_THREADS=$t timeout -k 10 200 python3 -u scripts/e2e_phases.py $c 21 2>&1 | grep -E "total|lower_end|run " || exit 1
  done
done
