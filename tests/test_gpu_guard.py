"""Bounded in-kernel waits (the slot protocol's forward-progress guard).

The dot products complete inside their producing kernels through
self-validating slots ("Dot completion"): a waiter spins until
the partials of blocks dispatched before it have arrived. HIP promises no
dispatch order, so every such wait is bounded ("spin_budget_us"). A wait that
outlives its budget writes a device error record and ends the solve; the call
returns HPCCG_HIP_EHIP naming the wait, and the next solve starts from emptied
slots. The debug option "dbg_withhold" withholds one slice's p.Ap partial so
the guard can be exercised: the solve must fail within the budget (not hang),
and the following solve must be bitwise the default one. The reference has no
such path: it aborts on a failed exchange (exchange_externals.cpp:119-125).
"""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BUDGET_US = 20000


def _solve(hp, M, n, max_iter=40):
    import torch
    b, _, _ = M.vectors()
    x = torch.zeros(n, dtype=torch.float64, device="cuda:0")
    _, it, nr, _ = hp.HPCCG(M, b, x, max_iter=max_iter, device=True)
    return it, nr, M.last_trace().tobytes(), x.cpu().numpy().tobytes()


CASES = {
    "direct_fused_update": (32, 32, 32, False, {}),
    "pairs_ring": (32, 32, 32, False, {"spmv_kernel": 2}),
    "direct_7pt": (24, 24, 40, True, {}),
    "eager": (32, 32, 32, False, {"use_graph": 0}),
    "unfused_update": (32, 32, 32, False, {"fuse_update": 0}),
}


@pytest.mark.parametrize("case", list(CASES))
def test_withheld_partial_times_out_then_recovers(hp, gpu, case):
    nx, ny, nz, p7, opts = CASES[case]
    n = nx * ny * nz
    ref_m = hp.Matrix.generate(nx, ny, nz, use_7pt=p7)
    for k, v in opts.items():
        ref_m.set_option(k, v)
    ref = _solve(hp, ref_m, n)
    M = hp.Matrix.generate(nx, ny, nz, use_7pt=p7)
    for k, v in opts.items():
        M.set_option(k, v)
    assert M.get_option("spin_budget_us") == 1000000  # the default bound
    nslices = (n + 511) // 512
    M.set_option("spin_budget_us", BUDGET_US)
    M.set_option("dbg_withhold", nslices // 2 + 1)
    t0 = time.time()
    with pytest.raises(hp.HPCCGError, match="device wait timed out") as ei:
        _solve(hp, M, n)
    dt = time.time() - t0
    assert dt < 10.0, dt  # one budget per wait (later waits see the record and leave at once)
    assert "iteration 1" in str(ei.value) and "solve abandoned" in str(ei.value)
    # the same matrix, guard off: slots were reset, so bitwise the default solve
    M.set_option("dbg_withhold", 0)
    assert _solve(hp, M, n) == ref
    assert _solve(hp, M, n) == ref


def test_withheld_partial_in_rank_group(hp, gpu):
    """The in-process group (two z-slab ranks on one GPU): a withheld partial
    on member 1 fails the group solve; the next group solve is the default's."""
    import torch

    def run(Ms):
        xs = [torch.zeros(16 * 16 * 12, dtype=torch.float64, device="cuda:0") for _ in Ms]
        bs = [M.vectors()[0] for M in Ms]
        _, it, nr, _ = hp.group_HPCCG(Ms, bs, xs, max_iter=30)
        return it, nr, Ms[0].last_trace().tobytes(), [x.cpu().numpy().tobytes() for x in xs]

    ref = run(hp.group_generate(16, 16, 12, 2))
    Ms = hp.group_generate(16, 16, 12, 2)
    Ms[1].set_option("spin_budget_us", BUDGET_US)
    Ms[1].set_option("dbg_withhold", 2)
    with pytest.raises(hp.HPCCGError, match="rank 1: device wait timed out"):
        run(Ms)
    Ms[1].set_option("dbg_withhold", 0)
    assert run(Ms) == ref


def test_guard_options_validated(hp, gpu):
    M = hp.Matrix.generate(8, 8, 8)
    with pytest.raises(hp.HPCCGError):
        M.set_option("spin_budget_us", 0)
    with pytest.raises(hp.HPCCGError):
        M.set_option("dbg_withhold", 10 ** 6)
    M.set_option("graph_chunk", 7)
    # the fused update bakes the parity of k into each captured launch: even chunks
    assert M.get_option("graph_chunk") == (8 if M.get_option("fuse_update") else 7)
