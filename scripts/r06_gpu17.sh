#!/bin/bash
# Round 6, the final build: the whole GPU suite, smoke(), the driver's
# default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/r06_suite.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06_suite.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/r06_smoke.log 2>&1 || exit $?
tail -n 2 gpurun_out/r06_smoke.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/r06_bench_final.log 2>&1 || exit $?
grep '^{' gpurun_out/r06_bench_final.log | python3 -c "
import json,sys
r=json.loads(sys.stdin.readlines()[-1])
print('value', r['value'], 'ms', r['ms_per_step'], 'frac', r['roofline']['frac'], 'kernel', r['roofline']['kernel_ms'], 'cpu', r['cpu_baseline']['value'])
print('parity', r.get('parity_sample'))
print('legs', {k: (r[k] or {}).get('value') for k in ('trig_leaves', 'fp32', 'evolved', 'deep_core')})
print('side', {k: (v.get('kernel_ms'), v.get('e2e_ms')) for k, v in (r.get('side_configs') or {}).items() if isinstance(v, dict)})
print('cold', r['e2e']['cold'])"
