"""Option resident_update: the fused update run by the
resident pair kernel (k_spmv_ar: every pair unit of the launch resident, Ap
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
    assert M.get_option("fuse_update") == 1 and M.get_option("resident_update") == 0
    ref = _solve(hp, M, it, gpu)
    M.set_option("resident_update", 1)
    assert M.get_option("resident_update") == 1
    for graph in (1, 0):
        M.set_option("use_graph", graph)
        assert _solve(hp, M, it, gpu) == ref, (dims, graph)
    M.close()


def test_resident_update_falls_back_when_units_do_not_fit(hp, gpu):
    M = hp.Matrix.generate(200, 200, 40)  # 1563 pair units: more than the chip holds at once
    M.set_option("spmv_kernel", 1)
    ref = _solve(hp, M, 30, gpu)
    M.set_option("resident_update", 1)
    assert M.get_option("resident_update") == 0
    assert _solve(hp, M, 30, gpu) == ref
    M.close()


def test_resident_update_guard(hp, gpu):
    """A withheld p.Ap partial: the resident blocks' p.Ap wait gives up within
    the spin budget (EHIP) and the next solve is bitwise the first."""
    M = hp.Matrix.generate(40, 36, 30)
    M.set_option("resident_update", 1)
    ref = _solve(hp, M, 60, gpu)
    M.set_option("spin_budget_us", 100000)
    M.set_option("dbg_withhold", 3)
    with pytest.raises(hp.HPCCGError, match="timed out"):
        _solve(hp, M, 60, gpu)
    M.set_option("dbg_withhold", 0)
    assert _solve(hp, M, 60, gpu) == ref
    M.close()
