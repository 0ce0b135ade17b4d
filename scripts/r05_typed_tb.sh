#!/bin/bash
# round 5: typed target blocks 32768 (default) vs 65536: C5, C5 deep trees; typed tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "c5 or typed or spambase" > gpurun_out/tb_tests.log 2>&1
rc=$?; tail -1 gpurun_out/tb_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for tb in 32768 65536; do
    echo "== target $tb: $(GPE_TYPED_TARGET_BLOCKS=$tb timeout -k 10 300 python3 scripts/bench_configs.py --only c5,c5_deep --reps 5 2>&1 | grep '^{' | python3 -c "
import json,sys
print(' | '.join('%s %s %s' % (r['config'], r['kernel_ms'], r['e2e_ms']) for r in map(json.loads, sys.stdin)))")"
  done
done
