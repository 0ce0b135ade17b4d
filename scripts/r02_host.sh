#!/bin/bash
# C3 / C5 evaluate() breakdown at 1, 4 and 16 host threads (flattener).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in c3 c5; do
  for t in 1 4 16; do
    OMP_NUM_THREADS=$t DEAP_AMD_FLAT_TIMING=1 timeout -k 10 300 python -u scripts/e2e_breakdown.py $cfg \
      > gpurun_out/host_${cfg}_t$t.log 2>&1
    rc=$?; echo "$cfg t=$t rc=$rc"; grep -v amdgpu.ids gpurun_out/host_${cfg}_t$t.log | tail -4
    [ $rc -eq 0 ] || exit $rc
  done
done
nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)))"
