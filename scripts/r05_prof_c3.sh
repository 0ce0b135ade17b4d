#!/bin/bash
# round 5: kernel + copy trace of evaluate at pop 1M (C3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_c3 -o c3 -- python3 -u scripts/e2e_phases.py c3 5 > gpurun_out/prof_c3.log 2>&1
rc=$?; tail -12 gpurun_out/prof_c3.log; exit $rc
