#!/bin/bash
# A/B of interpreter variants on the bench workload (one GPU call).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { local tag=$1; shift; timeout -k 10 240 env "$@" > gpurun_out/ab_$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc"; grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"geometry": {[^}]*}' gpurun_out/ab_$tag.log | tr '\n' ' '; echo; return $rc; }
run asm python3 -u bench.py --no-cpu-baseline --steps 2 || exit 1
run asm_notrig python3 -u bench.py --no-cpu-baseline --steps 2 --no-trig || exit 1
run cpp_notrig GPE_ASM=0 python3 -u bench.py --no-cpu-baseline --steps 2 --no-trig || exit 1
exit 0
