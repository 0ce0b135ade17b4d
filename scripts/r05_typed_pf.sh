#!/bin/bash
# round 5: the typed core with END prefetching the next program's window
# (variant libgpeval_tpf.so, GEN_ASM_PF_TYPED=1) against the tree's library:
# C5 parity, then C5 at pop 1M
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
DEAP_AMD_LIB=deap_amd/libgpeval_tpf.so timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "c5 or typed or spambase" > gpurun_out/tpf_tests.log 2>&1
rc=$?; tail -1 gpurun_out/tpf_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for lib in deap_amd/libgpeval.so deap_amd/libgpeval_tpf.so; do
    echo "== $lib: $(DEAP_AMD_LIB=$lib timeout -k 10 200 python3 scripts/bench_configs.py --only c5 --reps 5 2>&1 | grep '^{' | python3 -c "
import json,sys; r=json.loads(sys.stdin.read()); print(r['kernel_ms'], r['e2e_ms'])")"
  done
done
