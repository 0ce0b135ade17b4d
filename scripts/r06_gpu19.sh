#!/bin/bash
# Round 6 measurement: the share of wave lifetime the exact core's waves wait
# at the per-tile block barrier (GPE_DIAG=32 on a diagnostic build,
# libgpeval_diag.so: clock reads around the barrier), at the tuned planner
# weights and without them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "tuned:" "w0:GPE_TRIG_W=0 GPE_DIV_W=0" "p5:GPE_ASM_P=5"; do
  tag=${spec%%:*}; envs=${spec#*:}
  timeout -k 10 240 env DEAP_AMD_LIB=deap_amd/libgpeval_diag.so GPE_DIAG=32 $envs \
    python3 -u bench.py --no-cpu-baseline --no-side-configs --no-trig-leaves --no-fp32 \
    --steps 1 --warmup 0 > gpurun_out/diag_$tag.log 2>&1 || exit $?
  echo "$tag: $(grep diag32 gpurun_out/diag_$tag.log | tail -n 1) | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/diag_$tag.log)"
done
