set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "integer_residual or exact_integer or tournament or communicator or lexicase or c1_symbreg or adf or harm" > gpurun_out/t_exact.log 2>&1; echo "pytest rc=$?"
tail -n 30 gpurun_out/t_exact.log
bash scripts/handler_ab.sh "base:DEAP_AMD_LIB=deap_amd/libgpeval_k2.so" "al5:DEAP_AMD_LIB=deap_amd/libgpeval_al5.so" "al6:DEAP_AMD_LIB=deap_amd/libgpeval_al6.so" "al7:DEAP_AMD_LIB=deap_amd/libgpeval_al7.so" && bash scripts/ab.sh "base:DEAP_AMD_LIB=deap_amd/libgpeval_k2.so" "al6:DEAP_AMD_LIB=deap_amd/libgpeval_al6.so" "al5:DEAP_AMD_LIB=deap_amd/libgpeval_al5.so"
