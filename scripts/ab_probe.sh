#!/bin/bash
# Same-box A/B: per variant the neg-chain probe (per node / per program) and
# the headline kernel time.  Usage: bash scripts/ab_probe.sh TAG "name:ENV=v ..." ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=$1; shift
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  timeout -k 10 120 env $envs python3 -u scripts/overhead_probe.py --shapes ${SHAPES:-add,pushv} --lengths 9,33,129 \
    > gpurun_out/${tag}_${name}_probe.jsonl 2>&1 || exit 1
  echo "$name $(grep fit gpurun_out/${tag}_${name}_probe.jsonl | tr '\n' ' ')"
  if [ -z "${NO_BENCH:-}" ]; then
    timeout -k 10 200 env $envs python3 -u bench.py --no-cpu-baseline --no-side-configs --no-fp32 \
      --no-trig-leaves --steps 2 > gpurun_out/${tag}_${name}_bench.log 2>&1 || exit 1
    python3 -c "
import json
r=json.loads([l for l in open('gpurun_out/${tag}_${name}_bench.log') if l.startswith('{')][-1])
p=r.get('parity_sample') or {}
print('$name', 'value', r['value'], 'kernel_ms', r['roofline']['kernel_ms'], 'parity', p.get('bit_identical'), p.get('failed'))"
  fi
done
