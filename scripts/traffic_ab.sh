#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE passes) of the C4 bench for a variant
# library: bash scripts/traffic_ab.sh <tag> <lib.so>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; lib=$2
out=gpurun_out/traffic_$tag
mkdir -p $out
args="--no-cpu-baseline --no-side-configs --no-trig-leaves --no-fp32 --steps 2 --warmup 1"
export DEAP_AMD_LIB=$lib
timeout -s KILL 240 rocprofv3 --output-format csv --pmc FETCH_SIZE -d $out/pmc3 -o run -- python3 bench.py $args > $out/pmc3.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --output-format csv --pmc WRITE_SIZE SQ_WAVES -d $out/pmc4 -o run -- python3 bench.py $args > $out/pmc4.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
