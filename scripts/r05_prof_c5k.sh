#!/bin/bash
# round 5: rocprofv3 kernel statistics of the C5 leg at pop 1M (typed core)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_c5k
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5k -o c5 -- python3 scripts/bench_configs.py --only c5 --reps 5 > gpurun_out/prof_c5k.log 2>&1 || exit 1
grep '^{' gpurun_out/prof_c5k.log | head -1 | cut -c1-200
