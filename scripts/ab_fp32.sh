#!/bin/bash
# Same-box A/B of the fp32 mode leg: bash scripts/ab_fp32.sh TAG name:lib.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=$1; shift
for spec in "$@"; do
  name=${spec%%:*}; lib=${spec#*:}
  DEAP_AMD_LIB=$lib timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-side-configs \
    --no-trig-leaves --steps 2 > gpurun_out/${tag}_${name}.log 2>&1 || exit 1
  python3 -c "
import json
r=json.loads([l for l in open('gpurun_out/${tag}_${name}.log') if l.startswith('{')][-1])
f=r['fp32']; print('$name', 'fp64', r['ms_per_step'], 'fp32', f['ms_per_step'], f['value'], 'evolved', r['evolved']['ms_per_step'], 'deep', r['deep_core']['ms_per_step'])"
done
