#!/bin/bash
# Round-2 GPU call: full GPU suite, then the redo-threshold A/B with the
# headline parity sample.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -v --timeout 250 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/gpu_tests.log | grep -v PASSED | head -20; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for e in 40 30 20; do
  GPE_REDO_EXP=$e timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fp32 --no-trig-leaves --steps 3 --warmup 1 > gpurun_out/redo_$e.log 2>&1
  rc=$?; echo "redo_exp=$e rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 - gpurun_out/redo_$e.log <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ps = r["parity_sample"]
print("  value %.1f kernel_ms %.2f redo %s tiles %s | parity max_rel %.3g bit_identical %d failed %s"
      % (r["value"], r["roofline"]["kernel_ms"], r["config"]["geometry"]["redo"],
         r["config"]["geometry"]["redo_tiles"], ps["max_rel"], ps["bit_identical"], ps["failed"]))
PY
done
