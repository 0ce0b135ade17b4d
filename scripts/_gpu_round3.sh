# round-3 scratch GPU session (see the calls in the session log)
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "exact or deep or parity or redo or golden" > gpurun_out/t_sel.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/t_sel.log | tail -n 15
[ $rc -eq 0 ] || exit $rc
bash scripts/ab.sh "base:" "xall:GPE_EXACT_ALL=1" || exit 1
HC_ARGS="" bash scripts/handler_ab.sh "exact:GPE_EXACT_ALL=1" || exit 1
bash scripts/trace_quick.sh q2
