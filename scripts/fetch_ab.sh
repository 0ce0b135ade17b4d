#!/bin/bash
# FETCH_SIZE (HBM/MALL reads) of the main evaluation kernel for two library
# builds: bash scripts/fetch_ab.sh <variant .so> (vs the in-tree library)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
args="--no-cpu-baseline --no-side-configs --no-trig-leaves --no-fp32 --steps 1 --warmup 0"
for tag in cur alt; do
  out=gpurun_out/fetch_$tag
  mkdir -p $out
  if [ $tag = alt ]; then export DEAP_AMD_LIB=$1; fi
  timeout -s KILL 240 rocprofv3 --output-format csv --pmc FETCH_SIZE -d $out -o run -- python3 bench.py $args > $out/log 2>&1
  rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find $out -name "run_counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
s = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "f_eval_asm<false, false, false>" in r["Kernel_Name"]:
        s[r["Dispatch_Id"]].append(float(r["Counter_Value"]))
for d, v in s.items():
    print("dispatch", d, "FETCH_SIZE KiB", sum(v), "-> GB (x2 gfx950)", sum(v) * 2048 / 1e9)
PY
done
