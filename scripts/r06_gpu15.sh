#!/bin/bash
# Round 6, the final build: rocprofv3 kernel trace + PMC passes of the bench
# workload (scripts/profile.sh r06b), then the driver's default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/profile.sh r06b || exit $?
timeout -k 10 600 python3 -u bench.py > gpurun_out/r06_bench_final.log 2>&1 || exit $?
grep '^{' gpurun_out/r06_bench_final.log | python3 -c "
import json,sys
r=json.loads(sys.stdin.readlines()[-1])
print('value', r['value'], 'ms', r['ms_per_step'], 'frac', r['roofline']['frac'], 'cpu', r['cpu_baseline']['value'])
print('parity', r.get('parity_sample'))"
