#!/bin/bash
# Per-handler cost (scripts/handler_cost.py) for several builds/settings in
# one GPU call:  bash scripts/handler_ab.sh "tag:ENV=val ENV2=val" ...
# Prints one line per variant: GPop/s per chain shape.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}
  timeout -k 10 200 env $envs python3 -u scripts/handler_cost.py ${HC_ARGS:-} \
      > gpurun_out/hc_$tag.log 2>&1 || { echo "$tag failed"; tail -n 5 gpurun_out/hc_$tag.log; exit 1; }
  python3 - "$tag" gpurun_out/hc_$tag.log <<'PY'
import json, sys
tag, path = sys.argv[1:]
recs = [json.loads(l) for l in open(path) if l.startswith("{")]
print("%-8s " % tag + " ".join("%s=%.0f" % (r["shape"], r["gpops"]) for r in recs))
PY
done
