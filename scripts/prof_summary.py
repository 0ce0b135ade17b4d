#!/usr/bin/env python3
"""Summarise a scripts/profile.sh run (rocprofv3 CSV output) as markdown.

Usage: python scripts/prof_summary.py gpurun_out/prof_<tag> [traffic.json]
           > profiles/<tag>.md

Per kernel: dispatches, mean duration (kernel trace), and every PMC counter
averaged per dispatch.  Derived lines for the interpreter kernel:
  * fp64 VALU utilisation = fp64 wave-instructions x 64 lanes / (CUs x 64
    lanes/clk x cycles), cycles = GRBM_GUI_ACTIVE (per-XCD counter: mean);
  * HBM read bytes = FETCH_SIZE (KiB) x 1024 x 2 — the MI355X guide's gfx950
    correction (FETCH_SIZE counts 64 B per 128 B wide read);
  * write bytes = WRITE_SIZE (KiB) x 1024;
  * VALU busy = SQ_INSTS_VALU x 4 clk (a wave64 VALU instruction holds a
    16-lane SIMD for 4 clocks) over 256 CU x 4 SIMD x cycles;
  * occupancy = SQ_WAVE_CYCLES x 4 (quad-cycles) / (CU x cycles) waves per
    CU, against the residency limit of the code object's VGPRs and the
    launch's LDS.
Registers, spills and LDS in the kernel headings come from the code object
(resources.txt, scripts/kernel_resources.sh), not from rocprofv3's
VGPR_Count column.  With a second argument, writes the traffic JSON bench.py
reports (the first fp64 f_eval_asm kernel).
"""
import json
import csv
import glob
import os
import sys
from collections import defaultdict

CU = 256
XCD = 8          # GRBM_GUI_ACTIVE is summed over the 8 XCDs


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0].replace("void ", "")


def resources(d):
    """kernel short name -> (vgpr, vgpr spill, sgpr, sgpr spill) from the
    code object notes (scripts/kernel_resources.sh output)."""
    out = {}
    path = os.path.join(d, "resources.txt")
    if not os.path.exists(path):
        return out
    for line in open(path):
        f = line.split()
        if len(f) < 9 or f[1] != "vgpr":
            continue
        out[f[0]] = (f[2], f[4], f[6], f[8])
    return out


def mangled_match(res, k):
    """Resource entry of a demangled kernel name: base name plus its
    template arguments mangled (bool Lb1E/Lb0E, int Li<n>E, double d,
    float f)."""
    base = k.split("<")[0].split("::")[-1]
    targs = k[len(k.split("<")[0]):].strip()
    key = base
    if targs.startswith("<"):
        m = []
        for a in targs.strip("<>").split(","):
            a = a.strip()
            m.append({"true": "Lb1E", "false": "Lb0E", "double": "d",
                      "float": "f"}.get(a, "Li%sE" % a))
        key = "%sI%sE" % (base, "".join(m))
    for name, v in res.items():
        if key in name:
            return v
    return None


def _probe(name, grid):
    """A one-wave base probe of an evaluation kernel (init_asm)."""
    return "f_eval_asm" in name and int(float(grid)) <= 64


def main(d, traffic_path=None):
    res = resources(d)
    bench = None
    blog = os.path.join(d, "bench_trace.log")
    if os.path.exists(blog):
        lines = [l for l in open(blog) if l.startswith("{")]
        bench = json.loads(lines[-1]) if lines else None
    traffic = None
    stats = list(csv.DictReader(open(os.path.join(d, "trace",
                                                  "run_kernel_stats.csv"))))
    # the evaluation kernels' one-wave base probes (gpe_create: each kernel
    # writes its core's handler table and address once) are not evaluation
    # dispatches: per-kernel averages from the trace without them
    tpath = os.path.join(d, "trace", "run_kernel_trace.csv")
    if os.path.exists(tpath):
        per = defaultdict(list)
        for r in csv.DictReader(open(tpath)):
            if _probe(r["Kernel_Name"], r["Grid_Size_X"]):
                continue
            per[r["Kernel_Name"]].append(int(r["End_Timestamp"]) -
                                         int(r["Start_Timestamp"]))
        total = sum(sum(v) for v in per.values()) or 1
        stats = [{"Name": k, "Calls": str(len(v)), "AverageNs": sum(v) / len(v),
                  "Percentage": "%.4g" % (100.0 * sum(v) / total)}
                 for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))]
    counters = defaultdict(lambda: defaultdict(list))
    meta = {}
    for f in sorted(glob.glob(os.path.join(d, "pmc*",
                                           "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if _probe(r["Kernel_Name"], r["Grid_Size"]):
                continue
            k = short(r["Kernel_Name"])
            counters[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = (r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"],
                       r["Grid_Size"], r["Workgroup_Size"])
    args = "--profile-only --steps 2 --warmup 1"
    if os.path.exists(os.path.join(d, "cmd.txt")):
        args = open(os.path.join(d, "cmd.txt")).read().strip()
    out = ["# rocprofv3 summary: %s" % os.path.basename(d.rstrip("/")), "",
           "Command: `rocprofv3 --kernel-trace --stats --output-format csv "
           "-- python3 bench.py %s` (warmup + timed dispatches of each "
           "evaluation kernel); PMC counters from separate `--pmc` passes "
           "(scripts/profile.sh)." % args, "",
           "## Kernel trace (--stats)", "",
           "| kernel | calls | avg ms | total % |", "|---|---|---|---|"]
    for r in stats:
        out.append("| %s | %s | %.3f | %s |" % (short(r["Name"]), r["Calls"],
                                               float(r["AverageNs"]) / 1e6,
                                               r["Percentage"]))
    out += ["", "## Counters (mean per dispatch)", ""]
    for k in sorted(counters, key=lambda k: -max(
            counters[k].get("SQ_WAVES", [0]))):
        c = counters[k]
        if max(c.get("SQ_WAVES", [0])) < 1000 or \
                max(c.get("GRBM_GUI_ACTIVE", [0])) < 8e7:
            continue
        m = meta[k]
        r = mangled_match(res, k)
        if r:
            out.append("### %s (code object: %s VGPRs, %s spilled, %s SGPRs, "
                       "%s SGPR spills to VGPR lanes; dynamic LDS %s B; grid "
                       "%s, block %s)" % ((k,) + r + m[2:]))
        else:
            out.append("### %s (VGPR %s, SGPR %s, LDS %s B, grid %s, block %s)"
                       % ((k,) + m))
        out.append("")
        mean = {n: sum(v) / len(v) for n, v in c.items()}
        for n in sorted(mean):
            out.append("* %s = %.4g" % (n, mean[n]))
        f64 = sum(mean.get(n, 0.0) for n in (
            "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64",
            "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64"))
        cyc = mean.get("GRBM_GUI_ACTIVE")
        if cyc:
            cyc /= XCD
            dur = [float(r["AverageNs"]) for r in stats
                   if short(r["Name"]) == k]
            if dur:
                out.append("* derived: %.4g GPU cycles per dispatch "
                           "(GRBM_GUI_ACTIVE / %d XCDs) = %.2f GHz over the "
                           "traced mean duration" % (cyc, XCD,
                                                      cyc / dur[0]))
        if f64 and cyc:
            out.append("* derived: fp64 VALU utilisation = %.1f%% "
                       "(%.3g fp64 wave-instr x 64 / (%d CU x 64 x %.4g clk))"
                       % (100 * f64 * 64 / (CU * 64 * cyc), f64, CU, cyc))
        f32 = sum(mean.get(n, 0.0) for n in (
            "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_ADD_F32",
            "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_TRANS_F32"))
        if f32 and cyc:
            out.append("* derived: fp32 VALU utilisation = %.1f%% "
                       "(%.3g fp32 wave-instr x 64 / (%d CU x 128 x %.4g clk))"
                       % (100 * f32 * 64 / (CU * 128 * cyc), f32, CU, cyc))
        if "SQ_INSTS_VALU" in mean and cyc:
            out.append("* derived: VALU busy = %.1f%% of SIMD cycles (every "
                       "VALU wave-instr x 4 clk over %d CU x 4 SIMD x cycles)"
                       % (100 * 4 * mean["SQ_INSTS_VALU"] / (CU * 4 * cyc), CU))
        if "SQ_WAVE_CYCLES" in mean and cyc:
            out.append("* derived: occupancy = %.1f waves per CU (SQ_WAVE_CYCLES"
                       " x 4 quad-cycles / (%d CU x cycles))"
                       % (4 * mean["SQ_WAVE_CYCLES"] / (CU * cyc), CU))
        if "SQ_LDS_BANK_CONFLICT" in mean and cyc:
            out.append("* derived: LDS bank-conflict cycles = %.1f%% of the "
                       "CU-cycles (%.3g over %d CU x %.4g clk)"
                       % (100 * mean["SQ_LDS_BANK_CONFLICT"] / (CU * cyc),
                          mean["SQ_LDS_BANK_CONFLICT"], CU, cyc))
        if "FETCH_SIZE" in mean:
            out.append("* derived: HBM read = %.1f MB per dispatch "
                       "(FETCH_SIZE x 1 KiB x 2, gfx950 correction)"
                       % (mean["FETCH_SIZE"] * 1024 * 2 / 1e6))
        if "WRITE_SIZE" in mean:
            out.append("* derived: HBM write = %.2f MB per dispatch"
                       % (mean["WRITE_SIZE"] * 1024 / 1e6))
        if traffic is None and k.startswith("f_eval_asm<false, false") and \
                "FETCH_SIZE" in mean and bench:
            nc = bench["config"]["node_evals_per_step"]
            traffic = {
                "kernel": k,
                "workload": {"pop": bench["config"]["pop"],
                             "cases": bench["config"]["cases"], "seed": 2024,
                             "min_depth": 4, "max_depth": 8, "world": 1},
                "fetch_bytes_per_launch": int(mean["FETCH_SIZE"] * 1024 * 2),
                "write_bytes_per_launch": int(mean.get("WRITE_SIZE", 0) * 1024),
                "algorithmic_bytes_per_launch": 101000000,
                "fp64_lane_ops_per_node_case": round(f64 * 64 / nc, 2),
                "fp64_issue_util": round(f64 * 64 / (CU * 64 * cyc), 3),
                "valu_busy": round(4 * mean["SQ_INSTS_VALU"] / (CU * 4 * cyc), 3),
                "occupancy_waves_per_cu": round(
                    4 * mean.get("SQ_WAVE_CYCLES", 0) / (CU * cyc), 1),
                "source": "profiles/%s.md: FETCH_SIZE x 1 KiB x 2 (gfx950 "
                          "correction) + WRITE_SIZE x 1 KiB of the main fp64 "
                          "f_eval_asm dispatch; rocprofv3 --pmc passes of "
                          "bench.py %s" % (os.path.basename(d.rstrip("/")),
                                           args)}
            traffic["traffic_bytes_per_launch"] = \
                traffic["fetch_bytes_per_launch"] + traffic["write_bytes_per_launch"]
        out.append("")
    print("\n".join(out))
    if traffic_path and traffic:
        with open(traffic_path, "w") as fh:
            json.dump(traffic, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
