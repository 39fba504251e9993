"""Degenerate starts and non-finite values through every launch form
(HPCCG.cpp:347-386, the loop test `normr > tolerance` at :358).

* A zero initial residual -- x0 = xexact (A 1 = b bitwise, KAT-1) or b = 0
  with x0 = 0 -- runs no iteration: niters 0, normr 0, x untouched.
* A negative tolerance from a zero residual takes the reference's 0/0 path:
  at k = 1 p = r = 0, alpha = 0/0 = NaN, so x and r turn NaN; k = 2 still
  runs (its test reads k = 1's normr, 0); the loop test is false for NaN at
  k = 3: niters 2, normr NaN, every x NaN.
* A NaN in b or x0 makes r0.r0 NaN: no iteration, normr NaN, x untouched.
* An infinite x0 entry (an interior row, a face row): the reference forms
  p = x + 0.0 x (HPCCG.cpp:347 through waxpby.cpp:77), NaN there, so r0.r0 is
  NaN and no iteration runs -- the prologue here must do the same (a plain
  copy would give +-inf rows and r0.r0 = inf, and the SELL-512-A holes of face
  rows, 0.0 times an infinite neighbour, NaN rows the reference does not have).
* An infinite b entry: r0.r0 = inf > 0, k = 1 forms p = r + 0.0 r (NaN at
  that row) and the NaN path ends at niters 2.

NaN partials travel through the self-validating dot slots (kSlotEmpty is a
signalling-NaN payload no arithmetic produces, compared bitwise), so no wait
may expire. The bar is the oracle (HPCCG.cpp restated, pinned to the
reference build on these same cases by
tests/test_oracle.py::test_degenerate_starts_match_reference): equal niters,
normr bitwise (or both NaN), x bitwise with NaN where the oracle's is NaN.
"""
import math

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

FORMS = {
    "persistent": ((40, 36, 30), False, {}),
    "resident": ((40, 36, 30), False, {"resident_update": 1}),
    "launches": ((40, 36, 30), False, {"resident_update": 0}),
    "eager": ((40, 36, 30), False, {"resident_update": 0, "use_graph": 0}),
    "pair": ((40, 36, 30), False, {"resident_update": 0, "spmv_kernel": 2}),
    "direct": ((40, 36, 30), False, {"resident_update": 0, "spmv_kernel": 1}),
    "unfused": ((40, 36, 30), False, {"resident_update": 0, "fuse_update": 0, "fuse_p": 0}),
    "fold0": ((40, 36, 30), False, {"resident_update": 0, "fold": 0}),
    "7pt": ((32, 32, 32), True, {}),
    "big": ((160, 160, 80), False, {}),  # no persistent launch: the per-iteration pair-ring kernel
}


def cases(A, rows):
    """(name, b, x0, max_iter, tolerance) on the oracle matrix A; rows: where
    the infinite entries go."""
    n = A.nrow
    out = [("exact", A.b, np.ones(n), 30, 0.0),
           ("zero_rhs", np.zeros(n), np.zeros(n), 30, 0.0),
           ("exact_negtol", A.b, np.ones(n), 30, -1.0)]
    b = A.b.copy()
    b[n // 3] = np.nan
    out.append(("nan_b", b, np.zeros(n), 30, 0.0))
    x0 = np.zeros(n)
    x0[n // 2 + 7] = np.nan
    out.append(("nan_x0", A.b, x0, 30, 0.0))
    for tag, i in rows.items():
        x0 = np.zeros(n)
        x0[i] = np.inf
        out.append((f"inf_x0_{tag}", A.b, x0, 30, 0.0))
        b = A.b.copy()
        b[i] = -np.inf
        out.append((f"inf_b_{tag}", b, np.zeros(n), 30, 0.0))
    return out


def stencil_rows(nx, ny, nz):
    mid = (nz // 2) * nx * ny + (ny // 2) * nx
    return {"interior": mid + nx // 2, "face": mid + nx - 1}


def same(got, ref):
    it, nr, x = got
    assert it == ref["niters"]
    assert (math.isnan(nr) and math.isnan(ref["normr"])) or nr == ref["normr"], (nr, ref["normr"])
    assert np.array_equal(x, ref["x"], equal_nan=True)


def _solve(hp, M, b, x0, max_iter, tol, gpu):
    import torch
    bt = torch.from_numpy(np.ascontiguousarray(b)).to(gpu)
    xt = torch.from_numpy(np.ascontiguousarray(x0)).to(gpu)
    _, it, nr, _ = hp.HPCCG(M, bt, xt, max_iter=max_iter, tolerance=tol, device=True)
    return it, nr, xt.cpu().numpy()


@pytest.mark.parametrize("form", list(FORMS))
def test_degenerate_starts(hp, gpu, form):
    dims, seven, opts = FORMS[form]
    M = hp.Matrix.generate(*dims, use_7pt=seven)
    for k, v in opts.items():
        M.set_option(k, v)
    A = oracle.generate(*dims, use_7pt=seven)
    for name, b, x0, mi, tol in cases(A, stencil_rows(*dims)):
        ref = oracle.hpccg(A, b=b, x=x0, max_iter=mi, tolerance=tol)
        got = _solve(hp, M, b, x0, mi, tol, gpu)
        try:
            same(got, ref)
        except AssertionError as e:
            raise AssertionError(f"{form}/{name}: {e}") from None
        if name == "exact_negtol":
            assert got[0] == 2 and np.isnan(got[2]).all()
    # nothing carried: a regular solve afterwards is bitwise a fresh matrix's
    ref = oracle.hpccg(A, max_iter=40)
    got = _solve(hp, M, A.b, np.zeros(A.nrow), 40, 0.0, gpu)
    assert got[0] == ref["niters"]
    M2 = hp.Matrix.generate(*dims, use_7pt=seven)
    for k, v in opts.items():
        M2.set_option(k, v)
    fresh = _solve(hp, M2, A.b, np.zeros(A.nrow), 40, 0.0, gpu)
    assert got[0] == fresh[0] and got[1] == fresh[1] and np.array_equal(got[2], fresh[2])
    if opts.get("resident_update", -1) != 0 and not seven:
        assert M.get_option("resident_retries") == 0
    M.close()
    M2.close()


def test_degenerate_starts_sell_csr(hp, gpu):
    """The SELL-512 kernel (a ragged CSR matrix, no A image, padding slots
    with column -1)."""
    from test_gpu_parity import _random_sym
    n = 1500
    row_ptr, cols, vals = _random_sym(n, 11)
    M = hp.Matrix.from_csr(row_ptr, cols, vals)
    assert M.get_option("has_a") == 0
    b = oracle.sparsemv(oracle.CSR(row_ptr, cols, vals, np.zeros(n), np.zeros(n), np.ones(n)), np.ones(n))
    A = oracle.CSR(row_ptr, cols, vals, np.zeros(n), b, np.ones(n))
    for name, bb, x0, mi, tol in cases(A, {"row0": 0, "mid": n // 2}):
        ref = oracle.hpccg(A, b=bb, x=x0, max_iter=mi, tolerance=tol)
        try:
            same(_solve(hp, M, bb, x0, mi, tol, gpu), ref)
        except AssertionError as e:
            raise AssertionError(f"sell/{name}: {e}") from None
    M.close()


def test_degenerate_starts_group(hp, gpu):
    """A 2-rank in-process group (the multi-rank transport: all-reduced dots,
    halo exchange): the same outcomes as the oracle's serial solve of the
    z-stacked global problem -- exact here, since no iteration or only the
    NaN path runs."""
    import torch
    nx, ny, nz, P = 12, 10, 8, 2
    A = oracle.generate(nx, ny, nz * P)
    n = nx * ny * nz
    # the rows next to the slab boundary: rank 0's last plane, rank 1's first
    rows = {"lo_side": n - nx * ny // 2, "hi_side": n + nx * ny // 2 + nx - 1}
    for name, b, x0, mi, tol in cases(A, rows):
        ref = oracle.hpccg(A, b=b, x=x0, max_iter=mi, tolerance=tol)
        Ms = hp.group_generate(nx, ny, nz, P)
        bs = [torch.from_numpy(b[r * n:(r + 1) * n].copy()).to(gpu) for r in range(P)]
        xs = [torch.from_numpy(x0[r * n:(r + 1) * n].copy()).to(gpu) for r in range(P)]
        _, it, nr, _ = hp.group_HPCCG(Ms, bs, xs, max_iter=mi, tolerance=tol)
        x = np.concatenate([t.cpu().numpy() for t in xs])
        try:
            same((it, nr, x), ref)
        except AssertionError as e:
            raise AssertionError(f"group/{name}: {e}") from None
        for M in Ms:
            M.close()
