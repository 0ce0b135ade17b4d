cd "${GRAFT_REPO_ROOT}"
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rskip_tests.log 2>&1; rc=$?; tail -2 gpurun_out/rskip_tests.log; [ $rc -eq 0 ] || exit $rc
NO_BENCH= SHAPES=add bash scripts/ab_probe.sh rsk "rskip:X=1" "norskip:DEAP_AMD_LIB=deap_amd/libgpeval_norskip.so" "rskip2:X=1" "norskip2:DEAP_AMD_LIB=deap_amd/libgpeval_norskip.so"
