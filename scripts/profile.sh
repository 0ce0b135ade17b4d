#!/bin/bash
# rocprofv3 kernel trace + stats and separate PMC passes for bench.py.
# Usage: bash scripts/profile.sh <tag> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r01}; shift
args=${BENCH_ARGS:-"--no-cpu-baseline --no-side-configs --no-trig-leaves --no-fp32 --steps 2 --warmup 1"}
out=gpurun_out/prof_$tag
mkdir -p $out
echo "$args" > $out/cmd.txt
bash scripts/kernel_resources.sh > $out/resources.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py $args > $out/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $out/pmc1 -o run -- python3 bench.py $args > $out/pmc1.log 2>&1
rc=$?; echo "pmc1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --output-format csv --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $out/pmc2 -o run -- python3 bench.py $args > $out/pmc2.log 2>&1
rc=$?; echo "pmc2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --output-format csv --pmc FETCH_SIZE -d $out/pmc3 -o run -- python3 bench.py $args > $out/pmc3.log 2>&1
rc=$?; echo "pmc3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --output-format csv --pmc WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 -d $out/pmc4 -o run -- python3 bench.py $args > $out/pmc4.log 2>&1
rc=$?; echo "pmc4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --output-format csv --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $out/pmc5 -o run -- python3 bench.py $args > $out/pmc5.log 2>&1
rc=$?; echo "pmc5 rc=$rc"
find $out -name "*.csv" | head -20
exit 0
