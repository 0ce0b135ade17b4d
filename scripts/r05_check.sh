#!/bin/bash
# round 5: the GPU suite and the default bench line on the current build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
  > gpurun_out/r05_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r05_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r05_smoke.log
timeout -k 10 900 python3 -u bench.py > gpurun_out/r05_bench_final.log 2>&1
echo "bench rc=$?"
grep "^{" gpurun_out/r05_bench_final.log | python3 -c "
import json,sys
r=json.loads(sys.stdin.readline()); print(r['value'], r['ms_per_step'], r['roofline']['frac'], r['roofline']['traffic'], r['config']['geometry'], r.get('parity_sample',{}).get('bit_identical'))"
