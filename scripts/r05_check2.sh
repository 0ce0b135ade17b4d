#!/bin/bash
# round 5: GPU suite, then the bench line (side configs: C2/C3/C5 e2e)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
  > gpurun_out/r05_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/r05_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u bench.py > gpurun_out/r05_bench_final.log 2>&1
echo "bench rc=$?"
grep "^{" gpurun_out/r05_bench_final.log | python3 -c "
import json,sys
r=json.loads(sys.stdin.readline()); print(r['value'], r['ms_per_step'], r['roofline']['frac'])
for k,v in r.get('side_configs',{}).items(): print(k, {a:b for a,b in v.items() if 'ms' in a})"
