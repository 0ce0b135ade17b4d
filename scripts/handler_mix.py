#!/usr/bin/env python3
"""Static instruction mix of the fp64 asm core on the bench population.

Flattens the bench's C4 population (seed 2024, genHalfAndHalf(4, 8), 65,536
trees) on the host, maps every word to its handler as translate_program
(gpeval.hip) does (RELOAD words included), counts the instructions of each
handler's fast path in gp_asm_core.inc, and prints the expected per-wave
instruction counts per node-case class: fp64 VALU, other VALU, SALU, LDS,
branch.  Compare with the rocprofv3 PMC counts (profiles/r02_*.md).

    python scripts/handler_mix.py [--pop N]
"""
import argparse
import collections
import os
import re
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from deap_amd import configs  # noqa: E402
from deap_amd.flatten import Flattener, Op  # noqa: E402

CORE = os.path.join(REPO, "deap_amd", "csrc", "gp_asm_core.inc")
FAMS = ["add", "sub", "rsub", "mul", "div", "rdiv", "ndiv", "nrdiv"]
WINDOW = 16


def parse_core():
    lines = []
    for l in open(CORE):
        m = re.match(r'\s*"(.*)\\n" \\$', l)
        if m:
            lines.append(m.group(1))
    return lines


def classify(ins):
    op = ins.split()[0]
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_load"):
        return "smem"
    if op in ("s_setpc_b64", "s_branch") or op.startswith("s_cbranch"):
        return "branch"
    if op.startswith("s_waitcnt") or op.startswith("s_nop"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        if "_f64" in op and not op.startswith(("v_cmp", "v_cndmask")):
            return "fp64"
        return "valu"
    return "other"


def handler_costs(lines):
    """label -> Counter of the fast path (to the first s_setpc_b64; an
    s_branch to a shared body follows it)."""
    labels = {}
    for i, l in enumerate(lines):
        m = re.match(r"(\.L\w+?)_?%=:$", l)
        if m:
            labels[m.group(1)] = i
    out = {}
    for lab, i in labels.items():
        if not lab.startswith(".Lh_"):
            continue
        c = collections.Counter()
        j = i + 1
        while j < len(lines):
            l = lines[j]
            if l.endswith("%=:"):
                j += 1
                continue
            ins = l.split()[0]
            if ins == "s_branch" and ".Lbody" in l:
                j = labels[l.split()[1].replace("_%=", "").rstrip("_")]
                continue
            c[classify(l)] += 1
            if ins in ("s_setpc_b64", "s_branch"):
                break
            j += 1
        out[lab[4:].rstrip("_")] = c
    return out


def handler_name(op, d, x):
    if op == Op.LDV:
        return "LDV%d" % x
    if op == Op.LDC:
        return "LDC"
    if op == Op.PUSH:
        return "PUSH%d" % d
    if op == Op.PUSHV:
        return "PUSHV%d_%d" % (d, x)
    if op == Op.PUSHC:
        return "PUSHC%d" % d
    if op == Op.NEG:
        return "NEG"
    if op == Op.SIN:
        return "SIN"
    if op == Op.COS:
        return "COS"
    np_ = op >= Op.NPDIV
    fam = 6 + (op - Op.NPDIV) // 3 if np_ else (op - Op.ADD) // 3
    form = (op - Op.NPDIV) % 3 if np_ else (op - Op.ADD) % 3
    f = FAMS[fam]
    return ("%s_S%d" % (f, d), "%s_V%d" % (f, x), "%s_C" % f)[form]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pop", type=int, default=65536)
    ap.add_argument("--seed", type=int, default=2024)
    a = ap.parse_args()
    pset = configs.pset_for("symreg10")
    pop = configs.population(pset, "half", a.pop, a.seed, 4, 8)
    batch = Flattener(pset).flatten(pop)
    costs = handler_costs(parse_core())
    counts = collections.Counter()
    code, off = batch.code, batch.offsets
    for i in range(len(batch)):
        pos = 0
        j = int(off[i])
        while True:
            w = int(code[j])
            op, d, x = w & 0xff, (w >> 8) & 0xff, w >> 16
            j += 1
            if op == Op.END:
                counts["END"] += 1
                break
            konst = op in (Op.LDC, Op.PUSHC) or (
                op >= Op.ADD and op not in (Op.NEG, Op.SIN, Op.COS) and
                (op - (Op.NPDIV if op >= Op.NPDIV else Op.ADD)) % 3 == 2)
            need = 3 if konst else 1
            if pos + need > WINDOW - 1:
                counts["RELOAD"] += 1
                pos = 0
            counts[handler_name(op, d, x)] += 1
            pos += need
            if konst:
                j += 2
    nodes = int(batch.length.sum())
    tot = collections.Counter()
    groups = collections.defaultdict(collections.Counter)
    for h, n in counts.items():
        for k, v in costs[h].items():
            tot[k] += v * n
        g = re.sub(r"\d+(_\d+)?$", "", h)
        groups[g]["n"] += n
        for k, v in costs[h].items():
            groups[g][k] += v * n
    print("programs %d, reference nodes %d, handlers %d (%.3f per node)"
          % (len(batch), nodes, sum(counts.values()),
             sum(counts.values()) / nodes))
    print("%-10s %8s %7s | per handler: %6s %6s %6s %6s %6s | share of VALU"
          % ("handler", "count", "/node", "fp64", "valu", "salu", "lds",
             "branch"))
    allv = tot["fp64"] + tot["valu"]
    for g, c in sorted(groups.items(), key=lambda kv: -(kv[1]["fp64"] + kv[1]["valu"])):
        n = c["n"]
        print("%-10s %8d %7.3f | %19.1f %6.1f %6.1f %6.1f %6.1f | %5.1f%%"
              % (g, n, n / nodes, c["fp64"] / n, c["valu"] / n, c["salu"] / n,
                 c["lds"] / n, c["branch"] / n,
                 100.0 * (c["fp64"] + c["valu"]) / allv))
    print("per reference node (one wave = 128 node-cases): " + ", ".join(
        "%s %.2f" % (k, v / nodes) for k, v in sorted(tot.items())))
    print("fp64 share of VALU %.1f%%; fp64 lane-ops per node-case %.2f"
          % (100.0 * tot["fp64"] / allv, tot["fp64"] / nodes / 2))


if __name__ == "__main__":
    main()
