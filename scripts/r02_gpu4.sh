#!/bin/bash
# GPU suite, bench of the tree, and A/B of experimental library variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -v --timeout 250 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/gpu_tests.log | head -20; tail -2 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
summ() {
  python3 - "$1" <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ps = r.get("parity_sample") or {}
g = r["config"]["geometry"]
print("  value %.1f kernel_ms %.2f P %s groups %s redo %s tiles %s | parity max_rel %s bit_identical %s failed %s"
      % (r["value"], r["roofline"]["kernel_ms"], g["P"], g["groups"], g["redo"],
         g["redo_tiles"], ps.get("max_rel"), ps.get("bit_identical"), ps.get("failed")))
PY
}
for v in ${VARIANTS:-default}; do
  lib=""; [ "$v" = default ] || lib="DEAP_AMD_LIB=deap_amd/libgpeval_$v.so"
  env $lib ${VENV:-} timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fp32 --no-trig-leaves --steps 3 --warmup 1 > gpurun_out/ab_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  summ gpurun_out/ab_$v.log
done
