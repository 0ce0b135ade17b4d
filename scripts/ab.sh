#!/bin/bash
# A/B of evaluator variants on the bench workload (one GPU call).
# Usage: bash scripts/ab.sh "tag:ENV=val ENV2=val" ...   (default: a set)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  timeout -k 10 240 env "$@" python3 -u bench.py --no-cpu-baseline --steps 2 \
      ${AB_ARGS:-} > gpurun_out/ab_$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"geometry": {[^}]*}' gpurun_out/ab_$tag.log | tr '\n' ' ')"
  return $rc
}
if [ $# -eq 0 ]; then
  set -- "asm:GPE_ASM=1" "p6:GPE_ASM_P=6" "p4:GPE_ASM_P=4" "notrig:AB_DUMMY=1"
fi
for spec in "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}
  if [ "$tag" = notrig ]; then
    AB_ARGS="--no-trig" run $tag $envs || exit 1
  else
    run $tag $envs || exit 1
  fi
done
exit 0
