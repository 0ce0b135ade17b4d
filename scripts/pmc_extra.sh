#!/bin/bash
# Extra PMC passes on the bench workload: instruction cache and issue stalls.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
args="--no-cpu-baseline --no-side-configs --no-trig-leaves --no-fp32 --steps 1 --warmup 0"
out=gpurun_out/pmc_extra
mkdir -p $out
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $out/p1 -o run -- python3 bench.py $args > $out/p1.log 2>&1
echo "p1 rc=$?"
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQ_IFETCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $out/p2 -o run -- python3 bench.py $args > $out/p2.log 2>&1
echo "p2 rc=$?"
python3 - $out <<'PY'
import csv, glob, sys, collections
for f in sorted(glob.glob(sys.argv[1] + "/*/run_counter_collection.csv")):
    s = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "f_eval_asm<false, false, false>" in r["Kernel_Name"] and int(float(r["Grid_Size"])) > 64:
            s[r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in sorted(s.items()):
        print(k, "%.4g" % v)
PY
