#!/bin/bash
# round 5: kernel + copy trace of evaluate at pop 1M (C5), and its laps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_c5 -o c5 -- python3 -u scripts/e2e_phases.py c5 5 > gpurun_out/prof_c5.log 2>&1 || exit 1
GPE_DIAG=1 timeout -k 10 200 python3 -u scripts/e2e_phases.py c5 3 > gpurun_out/diag5_c5.log 2>&1 || exit 1
tail -40 gpurun_out/diag5_c5.log
