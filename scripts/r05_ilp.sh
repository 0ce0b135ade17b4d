#!/bin/bash
# round 5: the two chains interleaved in reduce_sincos and TAYLOR_SIN (variant build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DEAP_AMD_LIB=deap_amd/libgpeval_ilp.so timeout -k 10 240 python -u -m pytest tests/test_gpu.py -m gpu -v \
  -k "exact_asm_core or bench_hard or bench_sample or deep_asm_core" --timeout 200 --timeout-method thread \
  > gpurun_out/r05_ilp_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_ilp_tests.log; [ $rc -eq 0 ] || exit $rc
export AB_ARGS="--no-fp32"
bash scripts/ab.sh "base:X=1" "ilp:DEAP_AMD_LIB=deap_amd/libgpeval_ilp.so" "base2:X=2" \
  "ilp2:DEAP_AMD_LIB=deap_amd/libgpeval_ilp.so"
