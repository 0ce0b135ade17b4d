#!/bin/bash
# Redo policy A/B: threshold exponent x (pair list | whole programs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fp32 --no-trig-leaves --steps 3 --warmup 1 > gpurun_out/redo_$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 - gpurun_out/redo_$tag.log <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ps = r["parity_sample"]
g = r["config"]["geometry"]
print("  value %.1f kernel_ms %.2f P %s groups %s redo %s tiles %s | parity max_rel %.3g bit_identical %d failed %s"
      % (r["value"], r["roofline"]["kernel_ms"], g["P"], g["groups"], g["redo"],
         g["redo_tiles"], ps["max_rel"], ps["bit_identical"], ps["failed"]))
PY
}
run e40pairs GPE_REDO_EXP=40
run e40whole GPE_REDO_EXP=40 GPE_REDO_CAP=0
run e30pairs GPE_REDO_EXP=30
run e20pairs GPE_REDO_EXP=20
run e30whole GPE_REDO_EXP=30 GPE_REDO_CAP=0
