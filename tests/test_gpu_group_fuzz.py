"""Seeded random sweep of the multi-rank path (in-process rank group on one
GPU, the multi-rank kernels and halo plan; see test_gpu_group.py): 2-5 z-slab
ranks with thin slabs (down to one plane per rank), 1-wide axes, both
stencils, random iteration counts and option sets. Each case is checked

* against the CPU oracle's serial solve of the z-stacked global problem
  (generate_matrix.cpp:225-229; test infrastructure): niters equal, rtrans
  within RTRANS_RTOL_MULTI above the cutoff, every rank's x within 1e-9
  relative of its rows of the global x;
* against the same group solved with the default options: bitwise equal.
"""
import numpy as np
import pytest

import oracle
from conftest import RTRANS_RTOL_MULTI, check_trace

pytestmark = pytest.mark.gpu

SEED = 1600
CASES = 48
OPTIONS = {
    "spmv_kernel": (0, 1, 2, -1),
    "fuse_p": (0, -1),
    "fold": (0, 1, -1),
    "x_defer": (0, 1, 2),
    "x_ring": (2, 4, 8, 32, -1),
    "use_graph": (0, 1),
    "a2_ring": (-1, 0, 3),
}


def _cases():
    rng = np.random.default_rng(SEED)
    out = []
    for i in range(CASES):
        P = int(rng.integers(2, 6))
        s7 = bool(rng.integers(2))
        nx, ny = (int(v) for v in rng.integers(1, 17, size=2))
        nz = int(rng.integers(1, 9))
        max_iter = int(rng.integers(1, 61))
        opts = {k: int(rng.choice(v)) for k, v in OPTIONS.items()}
        out.append((i, P, (nx, ny, nz), s7, max_iter, opts))
    return out


def _solve(hp, Ms, max_iter):
    import torch
    xs = [torch.zeros(M.info()["nrow"], dtype=torch.float64, device="cuda:0") for M in Ms]
    bs = [M.vectors()[0] for M in Ms]
    ierr, niters, normr, _ = hp.group_HPCCG(Ms, bs, xs, max_iter=max_iter)
    assert ierr == 0
    return niters, normr, Ms[0].last_trace().copy(), [x.cpu().numpy() for x in xs]


@pytest.mark.parametrize("case", _cases(), ids=lambda c: f"c{c[0]}")
def test_random_groups(hp, gpu, case):
    _, P, (nx, ny, nz), s7, max_iter, opts = case
    hp.set_keep_sell(True)
    try:
        Ms = hp.group_generate(nx, ny, nz, P, use_7pt=s7)
    finally:
        hp.set_keep_sell(False)
    try:
        base = _solve(hp, Ms, max_iter)
        applied = {}
        for k, v in opts.items():
            prev = [M.get_option(k) for M in Ms]
            try:
                for M in Ms:
                    M.set_option(k, v)
                applied[k] = v
            except hp.HPCCGError:  # not available on some slab (e.g. no uniform width): all keep theirs
                for M, pv in zip(Ms, prev):
                    M.set_option(k, pv)
        got = _solve(hp, Ms, max_iter)
        for M in Ms[1:]:
            assert np.array_equal(M.last_trace(), got[2])  # one set of all-reduced scalars
    finally:
        for M in Ms:
            M.close()
    assert got[0] == base[0] and got[1] == base[1], (applied, got[:2], base[:2])
    assert got[2].tobytes() == base[2].tobytes(), applied
    assert all(a.tobytes() == b.tobytes() for a, b in zip(got[3], base[3])), applied
    A = oracle.generate(nx, ny, P * nz, use_7pt=s7)
    ref = oracle.hpccg(A, max_iter=max_iter)
    assert got[0] == ref["niters"], (applied, got[0], ref["niters"])
    check_trace(got[2], ref["trace"], RTRANS_RTOL_MULTI)
    x = np.concatenate(got[3])
    scale = max(1.0, float(np.max(np.abs(ref["x"]))))
    assert float(np.max(np.abs(x - ref["x"]))) <= 1e-9 * scale, applied
