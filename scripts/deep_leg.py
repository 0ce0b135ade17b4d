#!/usr/bin/env python3
"""bench.py's deep-core leg alone (one JSON line): the deep asm core and its
redo pass on tests/golden/c4_deep_core's trees x 16 at 2^20 C4 cases."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from deap_amd import datasets  # noqa: E402

X, y = datasets.symreg10_cases(2 ** 20, 2024)
print(json.dumps(bench.deep_core_leg(X, y, 2, 0)), flush=True)
