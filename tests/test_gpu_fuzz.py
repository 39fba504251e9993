"""Seeded random sweep of grid shapes, stencils, iteration counts, tolerances
and solver options on the HIP path (C ABI), each case checked two ways:

* against the CPU oracle (test infrastructure; oracle/hpccg_oracle.c, pinned to
  the reference): niters equal, rtrans within RTRANS_RTOL_1GPU above the
  cutoff, x within 1e-9 relative (the SpMV and waxpby are bitwise; the dots
  differ by association only);
* against the same matrix solved with the default options: bitwise equal
  (every option moves work, never a value).

Shapes include 1-wide axes, slice counts below and around the 8 XCDs and the
64-slice dot groups, odd pair counts, and early exits on a tolerance placed
between two of the oracle's residuals (never within rounding of either).
"""
import numpy as np
import pytest

import oracle
from conftest import RTRANS_RTOL_1GPU, check_trace

pytestmark = pytest.mark.gpu

SEED = 20261016
CASES = 64
# option -> values tried (-1 = the library's automatic choice)
OPTIONS = {
    "spmv_kernel": (0, 1, 2, -1),
    "fuse_p": (0, -1),
    "fold": (0, 1, -1),
    "x_defer": (0, 1, 2),
    "x_ring": (2, 3, 5, 8, 32, -1),
    "use_graph": (0, 1),
    "graph_chunk": (1, 3, 8, 32),
    "a2_ring": (-1, 0, 3),
    "fuse_update": (0, 1),
}


def _cases():
    rng = np.random.default_rng(SEED)
    out = []
    for i in range(CASES):
        s7 = bool(rng.integers(2))
        nx, ny = (int(v) for v in rng.integers(1, 25, size=2))
        nz = int(rng.integers(1, 41))
        max_iter = int(rng.integers(1, 91))
        early = bool(rng.integers(3) == 0)
        opts = {k: int(rng.choice(v)) for k, v in OPTIONS.items()}
        # the resident launches (the persistent one by default where it fits;
        # the per-iteration k_spmv_ar) against the other launch; drawn apart
        # so the cases above stay the seed's
        opts["resident_update"] = (0, -1, 1)[i % 3]
        out.append((i, (nx, ny, nz), s7, max_iter, early, opts))
    return out


def _solve(hp, M, b, max_iter, tol):
    x = np.zeros(len(b))
    ierr, it, nr, _ = hp.HPCCG(M, b, x, max_iter=max_iter, tolerance=tol)
    assert ierr == 0
    return it, nr, M.last_trace().copy(), x


@pytest.mark.parametrize("case", _cases(), ids=lambda c: f"c{c[0]}")
def test_random_shapes_and_options(hp, gpu, case):
    _, dims, s7, max_iter, early, opts = case
    hp.set_keep_sell(True)
    try:
        prob = hp.generate_matrix(*dims, use_7pt=s7)
        M = hp.Matrix.from_hpc(prob)
    finally:
        hp.set_keep_sell(False)
    A = oracle.generate(*dims, use_7pt=s7)
    ref = oracle.hpccg(A, max_iter=max_iter)
    tol = 0.0
    if early and ref["niters"] >= 3:
        # between two consecutive oracle residuals, above the rounding-noise
        # regime (normr >= 1e-9 normr0, where the traces agree to the 1e-8
        # bar): the loop test cannot flip on rounding
        tr = ref["trace"]
        above = int(np.sum(tr >= 1e-9 * tr[0]))  # the trace decreases: a leading run
        j = max(0, min(len(tr) - 2, above // 2))
        lo, hi = tr[j + 1], tr[j]
        if hi > 0 and lo > 1e-8 * hi and lo < 0.9 * hi:
            tol = float(np.sqrt(lo * hi))
            ref = oracle.hpccg(A, max_iter=max_iter, tolerance=tol)
    base = _solve(hp, M, prob.b, max_iter, tol)
    applied = {}
    for k, v in opts.items():
        try:
            M.set_option(k, v)
            applied[k] = v
        except hp.HPCCGError:  # not available for this matrix (e.g. no uniform width)
            pass
    got = _solve(hp, M, prob.b, max_iter, tol)
    M.close()
    # bitwise equal to the default-option solve
    assert got[0] == base[0] and got[1] == base[1], (applied, got[:2], base[:2])
    assert got[2].tobytes() == base[2].tobytes(), applied
    assert got[3].tobytes() == base[3].tobytes(), applied
    # the oracle
    assert got[0] == ref["niters"], (applied, got[0], ref["niters"])
    check_trace(got[2], ref["trace"], RTRANS_RTOL_1GPU)
    scale = max(1.0, float(np.max(np.abs(ref["x"]))))
    assert float(np.max(np.abs(got[3] - ref["x"]))) <= 1e-9 * scale, applied
