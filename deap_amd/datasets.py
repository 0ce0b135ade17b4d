"""Fitness-case sets of the five BASELINE configurations.

Each builder returns plain numpy arrays; the evaluator uploads them once and
keeps them resident in HBM.  Columns are stored variable-planar
(``X[var, case]``, contiguous over cases) — the layout the kernels stream.

* ``symbreg_points``  — ``examples/gp/symbreg.py:55-63``: 20 points ``x/10.``
  for x in [-10, 10), target terms ``x**4, x**3, x**2, x`` (Python ``**``).
* ``adf_symbreg_points`` — ``examples/gp/adf_symbreg.py:121-124``: the same
  20 points, one target column ``x**4 + x**3 + x**2 + x`` (Python).
* ``mux11_table``     — ``examples/gp/multiplexer.py:31-54`` truth table.
* ``parity6_table``   — ``examples/gp/parity.py:29-47`` truth table.
* ``symreg10_cases``  — synthetic 10-variable regression (config 4):
  X ~ U(-1, 1) from ``numpy.random.default_rng(seed)``, target
  ``deap/benchmarks/gp.py:60-72`` ``unwrapped_ball`` computed with Python's
  ``**`` (glibc ``pow``), which differs from ``d*d`` in ~1e-4 of rows.
* ``symbreg_numpy_points`` — ``examples/gp/symbreg_numpy.py:59-60``:
  ``numpy.linspace(-1, 1, 10000)`` and ``x**4 + x**3 + x**2 + x`` computed
  with numpy's own ``**`` and ``+`` (one target column).
* ``spambase_like``   — synthetic stand-in for ``examples/gp/spambase.csv``
  (4601 x 57 + label) matching the column statistics in SURVEY.md §8(d).
"""
import numpy as np

__all__ = ["symbreg_points", "symbreg_numpy_points", "adf_symbreg_points",
           "mux11_table",
           "parity6_table", "symreg10_cases", "spambase_like"]


def symbreg_points():
    """Returns ``(X[1, 20], terms[4, 20])`` (symbreg.py:55-63)."""
    pts = [x / 10. for x in range(-10, 10)]
    terms = [[x ** 4 for x in pts], [x ** 3 for x in pts],
             [x ** 2 for x in pts], list(pts)]
    return (np.array([pts], dtype=np.float64),
            np.array(terms, dtype=np.float64))


def adf_symbreg_points():
    """Returns ``(X[1, 20], target[1, 20])`` (adf_symbreg.py:121-124)."""
    pts = [x / 10. for x in range(-10, 10)]
    return (np.array([pts], dtype=np.float64),
            np.array([[x**4 + x**3 + x**2 + x for x in pts]],
                     dtype=np.float64))


def symbreg_numpy_points(n=10000):
    """Returns ``(X[1, n], values[1, n])`` (symbreg_numpy.py:59-60)."""
    samples = np.linspace(-1, 1, n)
    values = samples**4 + samples**3 + samples**2 + samples
    return samples[None, :], values[None, :]


def _bits_msb_first(n_bits):
    idx = np.arange(2 ** n_bits)
    return np.stack([(idx >> (n_bits - 1 - j)) & 1 for j in range(n_bits)])


def mux11_table():
    """``(inputs[11, 2048] in {0,1}, outputs[2048])`` — input line j of case i
    is bit (10-j) of i; output = data line ``3 + A0 + 2*A1 + 4*A2``
    (multiplexer.py:37-54)."""
    ins = _bits_msb_first(11)
    sel = 3 + ins[0] + 2 * ins[1] + 4 * ins[2]
    outs = ins[sel, np.arange(ins.shape[1])]
    return ins.astype(np.uint8), outs.astype(np.uint8)


def parity6_table():
    """``(inputs[6, 64], outputs[64])`` — output 1 for an even number of set
    inputs (parity.py:33-47)."""
    ins = _bits_msb_first(6)
    outs = 1 - (ins.sum(axis=0) & 1)
    return ins.astype(np.uint8), outs.astype(np.uint8)


def unwrapped_ball_py(X):
    """Row-wise ``10. / (5. + sum((d - 3)**2 for d in row))`` with Python
    semantics (``**`` is libm ``pow``; ``sum`` adds left to right)."""
    acc = np.zeros(X.shape[1], dtype=np.float64)
    for col in X:
        sq = np.fromiter(((d - 3) ** 2 for d in col.tolist()),
                         dtype=np.float64, count=col.shape[0])
        acc = acc + sq
    return 10. / (5. + acc)


def symreg10_cases(n_cases, seed=2024):
    """Config 4 data: ``(X[10, n], y[1, n])``."""
    rng = np.random.default_rng(seed)
    X = np.ascontiguousarray(rng.uniform(-1.0, 1.0, size=(n_cases, 10)).T)
    y = unwrapped_ball_py(X)
    return X, y[None, :]


def spambase_csv(path):
    """Config 5 on the reference's own data: ``examples/gp/spambase.csv``
    (4,601 rows of 57 features and a 0/1 label; gzip accepted), parsed as
    ``spambase.py:33-35`` parses it (``float`` of every field).  Returns
    ``(X[57, n], labels[n])``."""
    import csv
    import gzip
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rt") as fh:
        rows = [[float(v) for v in row] for row in csv.reader(fh)]
    A = np.asarray(rows, dtype=np.float64)
    if A.ndim != 2 or A.shape[1] != 58:
        raise ValueError("spambase rows have 58 fields")
    return np.ascontiguousarray(A[:, :57].T), (A[:, 57] != 0).astype(np.uint8)


def spambase_like(n_rows=4601, seed=1234):
    """Config 5 data: ``(X[57, n], labels[n] in {0,1})``.

    Columns 0-53: 81.7 % zeros, non-zeros lognormal (median 0.51, p99 ~7.5),
    rounded to 2 decimals; column 54: >=1, median ~2.3, 3 decimals;
    columns 55-56: integers >=1 with medians ~15 and ~95; label
    Bernoulli(0.394) — SURVEY.md §8(d) C5.
    """
    rng = np.random.default_rng(seed)
    X = np.zeros((57, n_rows), dtype=np.float64)
    nz = rng.random((54, n_rows)) >= 0.817
    vals = np.round(rng.lognormal(np.log(0.51), 1.156, size=(54, n_rows)), 2)
    X[:54] = np.where(nz, np.maximum(vals, 0.01), 0.0)
    X[54] = np.round(1.0 + rng.lognormal(np.log(1.3), 0.8, size=n_rows), 3)
    X[55] = np.floor(rng.lognormal(np.log(15.0), 0.9, size=n_rows)) + 1.0
    X[56] = np.floor(rng.lognormal(np.log(95.0), 1.1, size=n_rows)) + 1.0
    labels = (rng.random(n_rows) < 0.394).astype(np.uint8)
    return X, labels
