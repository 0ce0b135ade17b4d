#!/usr/bin/env python3
"""Golden for config 5 on the reference's own data: the rows of
``examples/gp/spambase.csv`` (4,601 x 58, read as ``spambase.py:33-35``
reads them) and typed programs of the reference's own primitive set, each
evaluated by the reference's ``gp.compile`` and the ``spambase.py:86``
expression — over ALL rows instead of ``random.sample(spam, 400)`` (the
declared deviation, SURVEY 8(a): the sample consumes the evolution's RNG and
is not reproducible).

Run in the build container only, against the 2to3 copy of the reference
(``make_oracle_copy.sh``); it imports the reference's ``examples/gp/
spambase.py`` module itself (its pset, its parsed rows) from that copy:

    bash tests/golden/make_oracle_copy.sh
    python3 tests/golden/_ref_spambase_real.py

Writes ``c5_spambase_real.json.gz`` (trees, hit counts) and
``spambase.csv.gz`` (the data file's rows, the fixture's inputs).
"""
import gzip
import hashlib
import json
import os
import random
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_COPY = os.environ.get("DEAP_ORACLE_COPY", "/tmp/deap_oracle")
CSV = "/root/reference/examples/gp/spambase.csv"


def main():
    sys.path.insert(0, ORACLE_COPY)
    ex = os.path.join(ORACLE_COPY, "examples", "gp")
    shutil.copy(CSV, os.path.join(ex, "spambase.csv"))
    cwd = os.getcwd()
    os.chdir(ex)                      # spambase.py opens "spambase.csv"
    sys.path.insert(0, ex)
    import spambase                   # the reference example (2to3 copy)
    from deap import gp
    os.chdir(cwd)
    pset, spam = spambase.pset, spambase.spam
    assert len(spam) == 4601 and all(len(r) == 58 for r in spam)

    def trees_of(seed, n, lo, hi):
        random.seed(seed)
        return [str(gp.PrimitiveTree(gp.genHalfAndHalf(pset, lo, hi)))
                for _ in range(n)]
    trees = trees_of(1501, 1000, 1, 2)          # spambase.py:75's generator
    trees += trees_of(1502, 300, 2, 6)
    # exact ties of the real rows: 81.7 % zeros, integer-valued columns
    # 55-56, repeated values; protectedDiv's int 1 against 1.0
    trees += ["eq(IN3, IN10)", "eq(IN0, IN1)", "eq(IN55, 1.0)",
              "eq(IN55, IN56)", "lt(IN55, IN56)", "lt(IN56, IN55)",
              "eq(protectedDiv(IN0, IN0), 1.0)",
              "eq(protectedDiv(IN4, IN7), protectedDiv(IN7, IN4))",
              "eq(sub(IN20, IN20), mul(IN31, 0.0))",
              "lt(IN54, 1.0)", "eq(IN54, 1.0)", "not_(eq(IN54, 1.0))",
              "eq(add(IN55, 1.0), IN56)", "eq(mul(IN55, 2.0), IN56)",
              "eq(IN26, IN27)", "and_(eq(IN0, 0.0), eq(IN1, 0.0))",
              "or_(lt(IN0, IN1), eq(IN0, IN1))",
              "eq(if_then_else(eq(IN0, 0.0), IN55, IN56), IN55)",
              "eq(protectedDiv(IN55, IN55), protectedDiv(IN56, IN56))",
              "lt(protectedDiv(IN5, 0.0), IN54)"]
    rows = [r[:57] for r in spam]
    labels = [r[57] for r in spam]
    hits = []
    for s in trees:
        func = gp.compile(s, pset)
        hits.append(int(sum(bool(func(*mail[:57])) is bool(mail[57])
                            for mail in spam)))
    flat = [v for r in spam for v in r]
    digest = hashlib.sha256(json.dumps(flat).encode()).hexdigest()
    with open(CSV, "rb") as src, open(os.path.join(HERE, "spambase.csv.gz"),
                                      "wb") as raw, \
            gzip.GzipFile(fileobj=raw, mode="wb", mtime=0) as dst:
        dst.write(src.read())
    out = {"pset": "spambase",
           "data": {"kind": "spambase_csv", "file": "spambase.csv.gz",
                    "rows": len(rows), "sha256_rows_json": digest},
           "source": "examples/gp/spambase.py (its pset and parsed rows) with "
                     "gp.compile and the spambase.py:86 expression over all "
                     "4,601 rows; trees from gp.genHalfAndHalf(1, 2) seed "
                     "1501, (2, 6) seed 1502, and tie cases",
           "trees": trees, "fitness": hits, "error": [None] * len(trees),
           "label_ones": int(sum(1 for v in labels if v))}
    with gzip.open(os.path.join(HERE, "c5_spambase_real.json.gz"), "wt") as fh:
        json.dump(out, fh)
    print("wrote c5_spambase_real.json.gz: %d trees" % len(trees))


if __name__ == "__main__":
    main()
