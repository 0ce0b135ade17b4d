#!/bin/bash
# Round-end measurements (usage: bash scripts/final.sh <tag> <stage>).  Stage "a": GPU suite, smoke, the default bench line.
# Stage "b": rocprofv3 trace + PMC passes.  Stage "c": per-shard scaling and
# per-config throughput.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-r04}
stage=${2:-a}
if [ "$stage" = a ]; then
  timeout -k 10 600 python -u -m pytest tests/ -m gpu -v --timeout 100 --timeout-method thread \
    > gpurun_out/${tag}_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/${tag}_tests.log | head -20; tail -2 gpurun_out/${tag}_tests.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  test_rc=$rc   # 1 = tests failed: smoke and bench still run, the call exits non-zero
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${tag}_smoke.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench_default.log 2>&1
  rc=$?; echo "bench rc=$rc"; grep "^{" gpurun_out/${tag}_bench_default.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
  if [ "$test_rc" -ne 0 ]; then echo "GPU tests FAILED (pytest rc=$test_rc)"; exit $test_rc; fi
  exit 0
fi
if [ "$stage" = b ]; then
  bash scripts/profile.sh $tag || exit 1
  exit 0
fi
for c in 1048576 524288 262144 131072; do
  timeout -k 10 200 python -u bench.py --cases $c --no-cpu-baseline --no-side-configs --no-fp32 --no-trig-leaves \
    --steps 5 --warmup 2 > gpurun_out/${tag}_shard_$c.log 2>&1
  rc=$?; echo "cases=$c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python -u scripts/bench_configs.py --reps 3 > gpurun_out/${tag}_configs.jsonl 2> gpurun_out/${tag}_configs.err
echo "configs rc=$?"
