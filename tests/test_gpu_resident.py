"""Option resident_update 1 (auto, -1, now picks the
persistent launch where it fits -- tests/test_gpu_persist.py): the fused
update run by the resident pair kernel (k_spmv_ar: every pair unit of the launch resident, Ap
and r kept in registers across the p.Ap completion, no Ap stream and no
second read of r). HPCCG.cpp:377-385 computed with the same expressions in
the same order as the default fused launch, so every solve must be bitwise
the default's; where the chip cannot hold every unit at once (200^3) the
option falls back to the default launch."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _solve(hp, M, it, gpu, b=None):
    import torch
    if b is None:
        b, _, _ = M.vectors()
    x = torch.zeros(M.info()["nrow"], dtype=torch.float64, device=gpu)
    _, n, nr, _ = hp.HPCCG(M, b, x, max_iter=it, device=True)
    return n, nr, M.last_trace().tobytes(), x.cpu().numpy().tobytes()


@pytest.mark.parametrize("dims,it", [((100, 100, 100), 90), ((40, 36, 30), 120), ((16, 16, 2), 40),
                                     ((64, 64, 64), 60)])
def test_resident_update_bitwise(hp, gpu, dims, it):
    M = hp.Matrix.generate(*dims)
    # the default here: the persistent launch (auto)
    assert M.get_option("fuse_update") == 1 and M.get_option("resident_update") == 8
    M.set_option("resident_update", 0)  # the unit + update-block launch
    assert M.get_option("resident_update") == 0
    ref = _solve(hp, M, it, gpu)
    M.set_option("resident_update", 1)
    assert M.get_option("resident_update") == 1
    for graph in (1, 0):
        M.set_option("use_graph", graph)
        assert _solve(hp, M, it, gpu) == ref, (dims, graph)
    M.set_option("resident_update", -1)
    assert _solve(hp, M, it, gpu) == ref, dims
    M.close()


def test_resident_update_falls_back_when_units_do_not_fit(hp, gpu):
    M = hp.Matrix.generate(200, 200, 40)  # 1563 pair units: more than the chip holds at once
    M.set_option("spmv_kernel", 1)
    M.set_option("resident_update", 0)
    ref = _solve(hp, M, 30, gpu)
    M.set_option("resident_update", 1)
    assert M.get_option("resident_update") == 0 and M.get_option("fuse_update") == 1
    assert _solve(hp, M, 30, gpu) == ref
    M.close()


def test_resident_update_guard(hp, gpu):
    """A withheld p.Ap partial: the resident blocks' p.Ap wait gives up within
    the spin budget (EHIP) and the next solve is bitwise the first."""
    M = hp.Matrix.generate(40, 36, 30)
    M.set_option("resident_update", 1)
    assert M.get_option("resident_update") == 1
    ref = _solve(hp, M, 60, gpu)
    M.set_option("spin_budget_us", 100000)
    M.set_option("dbg_withhold", 3)
    with pytest.raises(hp.HPCCGError, match="timed out"):
        _solve(hp, M, 60, gpu)
    M.set_option("dbg_withhold", 0)
    assert _solve(hp, M, 60, gpu) == ref
    M.close()


def test_resident_update_retry_on_expired_wait(hp, gpu):
    """A resident launch whose p.Ap wait expires -- what happens when another
    process holds part of the GPU and not every unit block can be resident;
    simulated by dbg_resident_stall -- is re-run from the caller's inputs with
    the unit + update-block launch: the call returns the default solve's
    bits, the retry is counted, and the matrix tries the resident launch
    again at its next solve (after three retries it keeps the other launch
    until switched back on)."""
    M = hp.Matrix.generate(40, 36, 30)
    M.set_option("resident_update", 1)
    ref = _solve(hp, M, 60, gpu)
    M.set_option("spin_budget_us", 50000)
    M.set_option("dbg_resident_stall", 1)
    assert _solve(hp, M, 60, gpu) == ref  # (the failed resident attempt, then the re-run)
    assert M.get_option("resident_retries") == 1 and M.get_option("resident_update") == 1
    assert _solve(hp, M, 60, gpu) == ref
    assert _solve(hp, M, 60, gpu) == ref
    assert M.get_option("resident_retries") == 3 and M.get_option("resident_update") == 0
    assert _solve(hp, M, 60, gpu) == ref
    M.set_option("dbg_resident_stall", 0)
    M.set_option("resident_update", 1)
    assert M.get_option("resident_update") == 1
    assert _solve(hp, M, 60, gpu) == ref
    # the host-pointer form re-stages the caller's x for the re-run too
    import numpy as np
    prob = hp.generate_matrix(40, 36, 30)
    H = hp.Matrix.from_hpc(prob)
    H.set_option("resident_update", 1)
    x0 = np.zeros(prob.nrow)
    _, n0, nr0, _ = hp.HPCCG(H, prob.b, x0, max_iter=60)
    H.set_option("spin_budget_us", 50000)
    H.set_option("dbg_resident_stall", 1)
    x1 = np.zeros(prob.nrow)
    _, n1, nr1, _ = hp.HPCCG(H, prob.b, x1, max_iter=60)
    assert (n1, nr1, x1.tobytes()) == (n0, nr0, x0.tobytes())
    H.close()
    M.close()
