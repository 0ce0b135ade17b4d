# round-3 scratch GPU session (see the calls in the session log)
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/t_all.log | tail -n 15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 > gpurun_out/bench_r3a.log 2> gpurun_out/bench_r3a.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_r3a.log
