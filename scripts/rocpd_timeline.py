#!/usr/bin/env python3
"""Kernel + copy timeline of the last evaluate in a rocprofv3 rocpd database
(rocprofv3 --kernel-trace --memory-copy-trace -d DIR -o NAME).  Usage:
python3 scripts/rocpd_timeline.py DB [anchor-kernel-substring] [n-anchors-back]"""
import sqlite3
import sys


def nm(n):
    n = n.replace('void ', '').replace('(anonymous namespace)::', '')
    n = n.replace('rocprim::ROCPRIM_400200_NS::detail::', '')
    return n.split('(')[0][:40]


def main():
    db = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "lower_trees"
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 7
    c = sqlite3.connect(db)
    ev = []
    for s, e, n, g, q in c.execute("select start,end,name,grid_x,stream_id from kernels"):
        ev.append((s, e, 'K s%s %s g%d' % (q, nm(n), g)))
    for s, e, n, sz, q in c.execute("select start,end,name,size,stream_id from memory_copies"):
        ev.append((s, e, 'C s%s %s %d' % (q, n, sz)))
    ev.sort()
    idx = [i for i, x in enumerate(ev) if anchor in x[2]]
    start = idx[-back]
    t0 = ev[start][0]
    j = start
    while j > 0 and ev[j - 1][0] > t0 - 1e6:
        j -= 1
    for s, e, n in ev[j:]:
        print("%8.3f %7.3f %s" % ((s - t0) / 1e6, (e - s) / 1e6, n))


if __name__ == "__main__":
    main()
