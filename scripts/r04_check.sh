#!/bin/bash
# GPU suite + default bench line + per-node/per-program probe (usage: r04_check.sh TAG)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-r04}
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/${tag}_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-side-configs --steps 3 > gpurun_out/${tag}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json,sys
r=json.loads([l for l in open('gpurun_out/${tag}_bench.log') if l.startswith('{')][-1])
print('value', r['value'], 'ms', r['ms_per_step'], 'kernel_ms', r['roofline']['kernel_ms'], 'parity', r.get('parity_sample',{}).get('bit_identical'), r.get('parity_sample',{}).get('failed'), 'max_rel', r.get('parity_sample',{}).get('max_rel'))
print('trig_leaves', r.get('trig_leaves',{}).get('value'), 'fp32', r.get('fp32',{}).get('value'))"
timeout -k 10 200 python -u scripts/overhead_probe.py --lengths 9,33,129 > gpurun_out/${tag}_overhead.jsonl 2>&1
rc=$?; grep fit gpurun_out/${tag}_overhead.jsonl; exit $rc
