"""Option resident_update -1 (auto; get_option reads 8): the persistent CG launch (k_cg_persist) --
every iteration after the prologue in ONE launch, each pair block holding its
rows' x in registers, the dots completed through per-iteration slots and
neighbour values read with sc1 loads. HPCCG.cpp:358-385 with the same
expressions in the same order as the per-iteration launches, so every solve
must be bitwise the default's (x, iteration count, residual trace)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _solve(hp, M, it, gpu, b=None, x0=None, tol=0.0):
    import torch
    if b is None:
        b, _, _ = M.vectors()
    n = M.info()["nrow"]
    x = torch.zeros(n, dtype=torch.float64, device=gpu) if x0 is None else x0.clone()
    _, niters, nr, _ = hp.HPCCG(M, b, x, max_iter=it, tolerance=tol, device=True)
    return niters, nr, M.last_trace().tobytes(), x.cpu().numpy().tobytes()


@pytest.mark.parametrize("dims,it", [((100, 100, 100), 90), ((40, 36, 30), 120), ((16, 16, 2), 40),
                                     ((64, 64, 64), 60), ((50, 50, 50), 50)])
def test_persistent_bitwise(hp, gpu, dims, it):
    M = hp.Matrix.generate(*dims)
    assert M.get_option("resident_update") == 8  # eligible: the persistent launch is the default here
    M.set_option("resident_update", 0)
    ref = _solve(hp, M, it, gpu)
    M.set_option("resident_update", -1)
    got = _solve(hp, M, it, gpu)
    assert M.get_option("resident_update") == 8 and M.get_option("resident_retries") == 0
    # the per-iteration resident launch (k_spmv_ar) too
    M.set_option("resident_update", 1)
    assert _solve(hp, M, it, gpu) == ref and M.get_option("resident_update") == 1
    M.set_option("resident_update", -1)
    assert got == ref, dims
    # a second solve on the same slots and buffers
    assert _solve(hp, M, it, gpu) == ref
    M.close()


def test_persistent_tolerance_exit_and_nonzero_x0(hp, gpu):
    """The loop test ends the launch part-way (tolerance reached), from a
    nonzero x0: same iteration count, trace and x as the default launches."""
    import torch
    M = hp.Matrix.generate(40, 36, 30)
    n = M.info()["nrow"]
    rng = np.random.default_rng(5)
    x0 = torch.from_numpy(rng.standard_normal(n)).to(gpu)
    b, _, _ = M.vectors()
    M.set_option("resident_update", 0)
    tr = np.frombuffer(_solve(hp, M, 100, gpu, b, x0)[2])
    tol = float(tr[60])  # the run stops at iteration 61 (normr <= tol there)
    ref = _solve(hp, M, 400, gpu, b, x0, tol)
    assert 50 < ref[0] < 80
    M.set_option("resident_update", -1)
    assert _solve(hp, M, 400, gpu, b, x0, tol) == ref
    M.close()


def test_persistent_max_iter_one(hp, gpu):
    M = hp.Matrix.generate(16, 16, 16)
    M.set_option("resident_update", 0)
    ref = [_solve(hp, M, it, gpu) for it in (1, 2, 3)]
    M.set_option("resident_update", -1)
    assert [_solve(hp, M, it, gpu) for it in (1, 2, 3)] == ref
    M.close()


def test_persistent_event_timing(hp, gpu):
    """Event timing (the bench's kernel clock) with the persistent launch:
    kernel_times covers the prologue and the launch, the solve is unchanged."""
    M = hp.Matrix.generate(40, 36, 30)
    M.set_option("resident_update", 0)
    ref = _solve(hp, M, 50, gpu)
    M.set_option("resident_update", -1)
    M.set_option("event_timing", 1)
    assert _solve(hp, M, 50, gpu) == ref
    kt = M.kernel_times()
    assert kt["spmv_ms"] > 0 and kt["spmv_launches"] == 50
    M.close()


def test_persistent_guard(hp, gpu):
    """A withheld p.Ap partial: the persistent launch's waits give up within
    the spin budget (EHIP, after the per-iteration re-run hits the same
    withheld partial) and the next solve is bitwise the first."""
    M = hp.Matrix.generate(40, 36, 30)
    M.set_option("resident_update", -1)
    ref = _solve(hp, M, 60, gpu)
    M.set_option("spin_budget_us", 100000)
    M.set_option("dbg_withhold", 3)
    with pytest.raises(hp.HPCCGError, match="timed out"):
        _solve(hp, M, 60, gpu)
    M.set_option("dbg_withhold", 0)
    M.set_option("resident_update", -1)
    assert _solve(hp, M, 60, gpu) == ref
    M.close()


def test_persistent_retry_on_expired_wait(hp, gpu):
    """A persistent launch whose wait expires (dbg_resident_stall: as when not
    every block can be resident) is re-run with the per-iteration launches:
    the caller gets the default solve's bits. Every retry is counted
    (resident_retries); the matrix tries the persistent launch again at its
    next solve until three retries have happened, then keeps the other launch."""
    M = hp.Matrix.generate(40, 36, 30)
    M.set_option("resident_update", 0)
    ref = _solve(hp, M, 60, gpu)
    M.set_option("resident_update", -1)
    M.set_option("spin_budget_us", 50000)
    M.set_option("dbg_resident_stall", 1)
    assert M.get_option("resident_retries") == 0
    assert _solve(hp, M, 60, gpu) == ref
    assert M.get_option("resident_retries") == 1 and M.get_option("resident_update") == 8  # re-armed
    assert _solve(hp, M, 60, gpu) == ref
    assert _solve(hp, M, 60, gpu) == ref
    assert M.get_option("resident_retries") == 3 and M.get_option("resident_update") == 0  # kept off now
    assert _solve(hp, M, 60, gpu) == ref
    assert M.get_option("resident_retries") == 3  # (no resident attempt any more)
    M.set_option("dbg_resident_stall", 0)
    M.set_option("resident_update", -1)  # switched back on by hand
    assert M.get_option("resident_update") == 8
    assert _solve(hp, M, 60, gpu) == ref
    assert M.get_option("resident_retries") == 3
    M.close()


def test_persistent_windows(hp, gpu):
    """A solve longer than one launch window (kPersistWindow = 512 iterations):
    the second launch resumes from the state the first left (x stored, the r.r
    history), bitwise the per-iteration launches -- to max_iter, and with a
    tolerance exit inside the second window."""
    M = hp.Matrix.generate(40, 36, 30)
    M.set_option("resident_update", 0)
    ref = _solve(hp, M, 1100, gpu)
    tr = np.frombuffer(ref[2])
    assert ref[0] > 700
    tol = float(tr[700])
    ref_tol = _solve(hp, M, 1100, gpu, tol=tol)
    assert 512 < ref_tol[0] < 1099
    M.set_option("resident_update", -1)
    assert M.get_option("resident_update") == 8
    assert _solve(hp, M, 1100, gpu) == ref
    assert _solve(hp, M, 1100, gpu, tol=tol) == ref_tol
    M.set_option("event_timing", 1)
    assert _solve(hp, M, 1100, gpu) == ref
    M.close()


@pytest.mark.parametrize("dims,it", [((3, 3, 3), 30), ((5, 7, 9), 60), ((101, 101, 101), 40)])
def test_persistent_edge_sizes(hp, gpu, dims, it):
    """The smallest shapes that take the persistent launch (one slice, a short
    odd slab) and the largest (101^3: 1008 pair blocks of the 1024 the chip
    holds at 4 per CU), bitwise the per-iteration launches."""
    M = hp.Matrix.generate(*dims)
    assert M.get_option("resident_update") == 8
    ref_default = _solve(hp, M, it, gpu)
    M.set_option("resident_update", 0)
    assert _solve(hp, M, it, gpu) == ref_default
    M.close()


def test_persistent_not_taken_beyond_the_chip(hp, gpu):
    """102^3 has more pair blocks (1061) than the chip holds at once: auto
    keeps the per-iteration launches (resident_update reads 0)."""
    M = hp.Matrix.generate(102, 102, 102)
    b, _, _ = M.vectors()
    import torch
    x = torch.zeros(102 ** 3, dtype=torch.float64, device=gpu)
    hp.HPCCG(M, b, x, max_iter=5, device=True)
    assert M.get_option("resident_update") == 0
    M.close()
