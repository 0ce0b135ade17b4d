#!/bin/bash
# round 5: evaluate phases and stamped laps at pop 1M (C5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python3 -u scripts/e2e_phases.py c5 21 2>&1 | grep -v amdgpu.ids || exit 1
GPE_DIAG=1 timeout -k 10 200 python3 -u scripts/e2e_phases.py c5 3 > gpurun_out/laps_c5.log 2>&1 || exit 1
grep -E "read_lower|gpe_lower_end|plan_mode|run_common|gpe_run|translate_device" gpurun_out/laps_c5.log | tail -22
