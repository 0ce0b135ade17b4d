#!/bin/bash
# round 5 records: kernel resources, rocprofv3 trace + PMC passes, the driver's bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/kernel_resources.sh > gpurun_out/r05_kernel_resources.txt 2>&1 || exit 1
bash scripts/profile.sh ${1:-r05c} || exit 1
timeout -k 10 900 python3 -u bench.py > gpurun_out/r05_bench_n1.log 2>&1
echo "bench rc=$?"
grep "^{" gpurun_out/r05_bench_n1.log | python3 -c "
import json,sys
r=json.loads(sys.stdin.readline()); print(r['value'], r['ms_per_step'], r['roofline']['frac'], r.get('parity_sample',{}).get('bit_identical'), (r.get('cpu_baseline') or {}).get('value'))"
