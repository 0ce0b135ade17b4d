#!/bin/bash
# A/B of evaluator variants on the bench workload (one GPU call).
# Usage: bash scripts/ab.sh "tag:ENV=val ENV2=val" ...
# Prints per variant: headline GPop/s, kernel ms, trig-leaf variant value.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  timeout -k 10 240 env "$@" python3 -u bench.py --no-cpu-baseline --no-side-configs --steps 2 \
      ${AB_ARGS:-} > gpurun_out/ab_$tag.log 2>&1
  local rc=$?
  python3 - "$tag" "$rc" gpurun_out/ab_$tag.log <<'PY'
import json, sys
tag, rc, path = sys.argv[1:]
line = [l for l in open(path) if l.startswith("{")]
if not line:
    print(tag, "rc=" + rc, "no JSON"); sys.exit()
r = json.loads(line[-1])
tl = r.get("trig_leaves") or {}
ps = r.get("parity_sample") or {}
print("%-10s rc=%s value=%.1f kernel_ms=%.1f | leaves value=%s kernel_ms=%s | "
      "parity max_rel=%s bit_identical=%s failed=%s | %s"
      % (tag, rc, r["value"], r["roofline"]["kernel_ms"], tl.get("value"),
         tl.get("kernel_ms"), ps.get("max_rel"), ps.get("bit_identical"),
         ps.get("failed"), r["config"]["geometry"]))
PY
  return $rc
}
for spec in "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}
  run $tag $envs || exit 1
done
exit 0
