#!/bin/bash
# The host stall at pop 1M: glibc trimming, Python's GC, or the
# device queue?  stall_probe.py under malloc tunables and GC modes, then a
# HIP-API + kernel timeline of the burst case.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local tag=$1; shift; timeout -k 10 240 env "$@" python3 -u scripts/stall_probe.py c5 burst,flat,free > gpurun_out/r04_stall_$tag.json 2>gpurun_out/r04_stall_$tag.err || exit 1; echo "$tag $(cat gpurun_out/r04_stall_$tag.json)"; }
run base X=1
run malloc MALLOC_TRIM_THRESHOLD_=17179869184 MALLOC_TOP_PAD_=1073741824 MALLOC_MMAP_THRESHOLD_=33554432
run gcfreeze STALL_GC=freeze
run gcoff STALL_GC=disable
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/r04_stall_trace -o run -- python3 scripts/stall_probe.py c5 burst > gpurun_out/r04_stall_trace.log 2>&1
echo "trace rc=$?"
