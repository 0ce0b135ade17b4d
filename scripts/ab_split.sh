cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
SHAPES=sin bash scripts/ab_probe.sh spl "base:X=1" "split:DEAP_AMD_LIB=deap_amd/libgpeval_split.so" "base2:X=1" "split2:DEAP_AMD_LIB=deap_amd/libgpeval_split.so" || exit 1
args="--no-cpu-baseline --no-side-configs --no-trig-leaves --no-fp32 --steps 1 --warmup 0"
for v in base split; do
  lib=""; [ $v = split ] && lib=deap_amd/libgpeval_split.so
  DEAP_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --output-format csv --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/spl_pmc_$v -o run -- python3 bench.py $args > gpurun_out/spl_pmc_$v.log 2>&1 || exit 1
  python3 - gpurun_out/spl_pmc_$v $v <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/run_counter_collection.csv")[0]
s = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(f)):
    if "f_eval_asm<false, false, false>" in r["Kernel_Name"] and int(float(r["Grid_Size"])) > 64:
        s[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
cyc = s["GRBM_GUI_ACTIVE"] / max(1, n["GRBM_GUI_ACTIVE"]) / 8
print(sys.argv[2], {k: "%.4g" % (v / max(1, n[k])) for k, v in s.items()},
      "conflict frac %.3f" % (s["SQ_LDS_BANK_CONFLICT"] / max(1, n["SQ_LDS_BANK_CONFLICT"]) / (256 * cyc)))
PY
done
