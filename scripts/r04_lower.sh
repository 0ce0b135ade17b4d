#!/bin/bash
# lower_trees on C3 at pop 1M: kernel trace + two PMC passes (usage: r04_lower.sh TAG)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r04}
out=gpurun_out/lower_$tag
mkdir -p $out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python3 scripts/lower_probe.py c3 5 > $out/trace.log 2>&1 || exit 1
grep lower_programs $out/trace.log | tail -3
f=$(find $out/trace -name "run_kernel_stats.csv" | head -1); grep -E "lower_trees|compact" "$f" | cut -d, -f1-4
if [ -n "${PMC:-}" ]; then
timeout -s KILL 120 rocprofv3 --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY \
  -d $out/p1 -o run -- python3 scripts/lower_probe.py c3 2 > $out/p1.log 2>&1; echo "p1 rc=$?"
timeout -s KILL 120 rocprofv3 --output-format csv --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR \
  -d $out/p2 -o run -- python3 scripts/lower_probe.py c3 2 > $out/p2.log 2>&1; echo "p2 rc=$?"
python3 - $out <<'PY'
import csv, glob, sys, collections
for f in sorted(glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv")):
    s = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "lower_trees" in r["Kernel_Name"]:
            s[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    for k, v in sorted(s.items()):
        print(k, "%.4g per dispatch" % (v / max(1, n[k] / 1)))
PY
fi
