"""Random sparse SPD systems through the CSR entry points (the Mode-2 /
drop-in path: any sparsity, entries in the caller's order), one rank and
split over 2-5 in-process ranks at random row boundaries, so the general
make_local_matrix plan (make_local_matrix.cpp:58-610: externals numbered by
owner in order of first appearance, requests exchanged, gathered sends) sees
ghost columns owned by non-adjacent ranks. Checked against the CPU oracle
(test infrastructure) on the same CSR: SpMV bitwise (entry order kept),
niters equal, rtrans within RTRANS_RTOL_1GPU (one rank) / RTRANS_RTOL_MULTI,
x within 1e-9 relative.
"""
import numpy as np
import pytest

import oracle
from conftest import RTRANS_RTOL_1GPU, RTRANS_RTOL_MULTI, check_final, check_trace

pytestmark = pytest.mark.gpu

SEED = 7


def random_spd(rng, n, per_row, band):
    """Symmetric, strictly diagonally dominant (so SPD), entries of each row in
    random order; b = A 1, x0 = 0 (like generate_matrix: xexact = 1)."""
    rows = [dict() for _ in range(n)]
    for i in range(n):
        for _ in range(int(rng.integers(0, per_row + 1))):
            j = int(i + rng.integers(-band, band + 1)) if band else int(rng.integers(0, n))
            if 0 <= j < n and j != i:
                v = -float(rng.uniform(0.05, 1.0))
                rows[i][j] = v
                rows[j][i] = v
    row_ptr = np.zeros(n + 1, np.int64)
    cols, vals = [], []
    for i in range(n):
        d = rows[i]
        ent = list(d.items()) + [(i, sum(-v for v in d.values()) + float(rng.uniform(0.5, 2.0)))]
        order = rng.permutation(len(ent))
        for k in order:
            cols.append(ent[k][0])
            vals.append(ent[k][1])
        row_ptr[i + 1] = len(cols)
    cols = np.asarray(cols, np.int32)
    vals = np.asarray(vals, np.float64)
    A = oracle.CSR(row_ptr, cols, vals, np.zeros(n), np.zeros(n), np.ones(n))
    A.b = oracle.sparsemv(A, np.ones(n))
    return A


def _cases(kind, count):
    rng = np.random.default_rng(SEED + (0 if kind == "single" else 1))
    out = []
    for i in range(count):
        n = int(rng.integers(1, 4000))
        per_row = int(rng.integers(0, 14))
        band = int(rng.choice([0, 1, 7, 300, 2000]))
        P = 1 if kind == "single" else int(rng.integers(2, 6))
        max_iter = int(rng.integers(1, 80))
        out.append((i, n, per_row, band, P, max_iter, int(rng.integers(1 << 30))))
    return out


def _check(ref, niters, normr, trace, x, rtol, max_iter):
    # small systems converge to rounding noise within max_iter: check_final's
    # termination rule (equal niters above the noise floor) applies
    check_final(niters, normr, trace, ref["niters"], ref["normr"], ref["trace"], max_iter)
    check_trace(trace, ref["trace"], rtol)
    scale = max(1.0, float(np.max(np.abs(ref["x"])))) if len(ref["x"]) else 1.0
    assert len(x) == len(ref["x"])
    if len(x):
        assert float(np.max(np.abs(x - ref["x"]))) <= 1e-9 * scale


@pytest.mark.parametrize("case", _cases("single", 16), ids=lambda c: f"c{c[0]}")
def test_random_csr_one_rank(hp, gpu, case):
    _, n, per_row, band, _, max_iter, seed = case
    A = random_spd(np.random.default_rng(seed), n, per_row, band)
    M = hp.Matrix.from_csr(A.row_ptr, A.cols, A.vals)
    try:
        # SpMV bitwise in the caller's entry order (HPC_sparsemv.cpp:76-87)
        import torch
        v = np.random.default_rng(seed + 1).uniform(-1, 1, n)
        y = torch.zeros(max(n, 1), dtype=torch.float64, device=gpu)
        hp.HPC_sparsemv(M, torch.from_numpy(v).to(gpu), y)
        assert y.cpu().numpy()[:n].tobytes() == oracle.sparsemv(A, v).tobytes()
        x = np.zeros(n)
        ierr, niters, normr, _ = hp.HPCCG(M, A.b, x, max_iter=max_iter)
        assert ierr == 0
        trace = M.last_trace().copy()
    finally:
        M.close()
    _check(oracle.hpccg(A, max_iter=max_iter), niters, normr, trace, x, RTRANS_RTOL_1GPU, max_iter)


@pytest.mark.parametrize("case", _cases("group", 16), ids=lambda c: f"c{c[0]}")
def test_random_csr_ranks(hp, gpu, case):
    import torch
    _, n, per_row, band, P, max_iter, seed = case
    rng = np.random.default_rng(seed)
    n = max(n, P)
    A = random_spd(rng, n, per_row, band)
    cuts = np.sort(rng.choice(np.arange(1, n), size=P - 1, replace=False)) if n > P else np.arange(1, P)
    bounds = [0] + [int(c) for c in cuts] + [n]
    parts = []
    for r in range(P):
        lo, hi = bounds[r], bounds[r + 1]
        rp = A.row_ptr[lo:hi + 1] - A.row_ptr[lo]
        parts.append((rp, A.cols[A.row_ptr[lo]:A.row_ptr[hi]], A.vals[A.row_ptr[lo]:A.row_ptr[hi]], lo))
    Ms = hp.group_from_csr(parts, n)
    try:
        bs = [torch.from_numpy(A.b[bounds[r]:bounds[r + 1]].copy()).to(gpu) for r in range(P)]
        xs = [torch.zeros(bounds[r + 1] - bounds[r], dtype=torch.float64, device=gpu) for r in range(P)]
        ierr, niters, normr, _ = hp.group_HPCCG(Ms, bs, xs, max_iter=max_iter)
        assert ierr == 0
        trace = Ms[0].last_trace().copy()
        for M in Ms[1:]:
            assert np.array_equal(M.last_trace(), trace)
        x = np.concatenate([t.cpu().numpy() for t in xs])
    finally:
        for M in Ms:
            M.close()
    _check(oracle.hpccg(A, max_iter=max_iter), niters, normr, trace, x, RTRANS_RTOL_MULTI, max_iter)
