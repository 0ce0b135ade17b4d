#!/bin/bash
# round 5: PMC counters of the typed core (C5 at pop 1M), two passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/typed_pmc
rm -rf $out
timeout -s KILL 120 rocprofv3 --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $out/pmc1 -o run -- python3 scripts/e2e_phases.py c5 1 > $out.p1.log 2>&1
rc=$?; echo "pmc1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --output-format csv --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $out/pmc2 -o run -- python3 scripts/e2e_phases.py c5 1 > $out.p2.log 2>&1
rc=$?; echo "pmc2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --output-format csv --pmc SQ_INSTS_VALU_FP64 SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM -d $out/pmc3 -o run -- python3 scripts/e2e_phases.py c5 1 > $out.p3.log 2>&1
rc=$?; echo "pmc3 rc=$rc"; exit $rc
