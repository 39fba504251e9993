"""Deterministic Mode-2 test systems (read_HPC_row.cpp format), no RNG.

general_system(n): a symmetric, strictly diagonally dominant (hence SPD)
matrix with couplings i +- 1, i +- 37, i +- 211 (mod n). Rows list their
entries in the order (i-211, i-37, i-1, i, i+1, i+37, i+211) mod n, so the wrap
rows are not sorted and, split over ranks, rank 0 needs columns from the last
rank: the z-slab halo plan cannot serve it and the gather plan
(make_local_matrix.cpp:58-610) must. x0 is nonzero (Mode 2 takes the initial
guess from the file), xexact = 1 and b = A * 1 summed in entry order.
All values are dyadic, so the file round-trips exactly through repr/strtod.
"""
import numpy as np

SHIFTS = (-211, -37, -1, 0, 1, 37, 211)


def general_system(n=600):
    assert n > 2 * 211 + 1
    rows_c, rows_v = [], []
    for i in range(n):
        cols = [(i + s) % n for s in SHIFTS]
        vals = []
        for c in cols:
            vals.append(0.0 if c == i else -1.0 - 0.125 * ((i + c) % 4))
        diag = sum(-v for v in vals) + 1.0 + 0.5 * (i % 3)
        vals[SHIFTS.index(0)] = diag
        rows_c.append(cols)
        rows_v.append(vals)
    row_ptr = np.zeros(n + 1, np.int64)
    row_ptr[1:] = np.cumsum([len(c) for c in rows_c])
    cols = np.array([c for r in rows_c for c in r], np.int32)
    vals = np.array([v for r in rows_v for v in r], np.float64)
    b = np.zeros(n)
    for i in range(n):
        s = 0.0
        for v in rows_v[i]:
            s = s + v * 1.0
        b[i] = s
    x0 = np.array([(i % 7) / 8.0 for i in range(n)])
    xexact = np.ones(n)
    return row_ptr, cols, vals, x0, b, xexact


def write(path, row_ptr, cols, vals, x, b, xexact):
    n = len(row_ptr) - 1
    with open(path, "w") as f:
        f.write(f"{n} {int(row_ptr[-1])}\n")
        for i in range(n):
            f.write(f"{int(row_ptr[i + 1] - row_ptr[i])}\n")
        for i in range(n):
            a, e = int(row_ptr[i]), int(row_ptr[i + 1])
            f.write(str(e - a) + " " + " ".join(f"{float(vals[k])!r} {int(cols[k])}" for k in range(a, e))
                    + "\n")
        for i in range(n):
            f.write(f"{float(x[i])!r} {float(b[i])!r} {float(xexact[i])!r}\n")
