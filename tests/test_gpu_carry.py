"""Nothing carries from one solve into the next.

HPCCG.cpp:342-356 starts every solve from r = b - A x; the device-resident
solver keeps iteration state, dot slots, ready slots, scalars and
rings between solves, and re-arms them at every solve start (k_rearm). Each
test solves one matrix with b1, then with b2 (a different right-hand side),
possibly after a disturbance -- the placement probe's timed solves and buffer
moves, an aborted solve (a withheld partial), option changes -- and requires
the b2 solve to be bitwise the b2 solve of a fresh matrix."""
import numpy as np
import pytest

from test_gpu_parity import DIRECT, PAIRS, SELL, keep_sell, solve_bits  # noqa: F401 (fixture)

pytestmark = pytest.mark.gpu

DIMS = (40, 36, 30)


def _rhs(prob):
    b1 = prob.b.copy()
    # b2: another right-hand side, not a multiple of b1
    i = np.arange(len(b1), dtype=np.float64)
    b2 = b1 * 0.5 + np.sin(i * 0.37)
    return b1, b2


def _fresh(hp, prob, kernel, b, it, opts=()):
    F = hp.Matrix.from_hpc(prob)
    F.set_option("spmv_kernel", kernel)
    for k, v in opts:
        F.set_option(k, v)
    out = solve_bits(hp, F, b, it)
    F.close()
    return out


@pytest.mark.parametrize("kernel,p7", [(DIRECT, False), (PAIRS, False), (DIRECT, True)])
@pytest.mark.parametrize("graph", [1, 0])
def test_back_to_back_rhs(hp, gpu, kernel, p7, graph):
    prob = hp.generate_matrix(*DIMS, use_7pt=p7)
    b1, b2 = _rhs(prob)
    opts = (("use_graph", graph),)
    want2 = _fresh(hp, prob, kernel, b2, 70, opts)
    want1 = _fresh(hp, prob, kernel, b1, 70, opts)
    M = hp.Matrix.from_hpc(prob)
    M.set_option("spmv_kernel", kernel)
    M.set_option("use_graph", graph)
    if kernel == DIRECT:
        assert M.get_option("fuse_update") == 1  # the one-launch iteration is the one exercised
    assert solve_bits(hp, M, b1, 70) == want1
    assert solve_bits(hp, M, b2, 70) == want2
    assert solve_bits(hp, M, b1, 70) == want1
    # a shorter solve, then the long one again (different max_iter: graph rebuilt)
    solve_bits(hp, M, b2, 9)
    assert solve_bits(hp, M, b2, 70) == want2
    M.close()


@pytest.mark.parametrize("kernel", [DIRECT, PAIRS])
def test_back_to_back_after_probe(hp, gpu, kernel):
    prob = hp.generate_matrix(*DIMS)
    b1, b2 = _rhs(prob)
    want2 = _fresh(hp, prob, kernel, b2, 60)
    M = hp.Matrix.from_hpc(prob)
    M.set_option("spmv_kernel", kernel)
    solve_bits(hp, M, b1, 60)
    M.probe_placement(2)
    assert solve_bits(hp, M, b2, 60) == want2
    M.close()


@pytest.mark.parametrize("kernel", [DIRECT, PAIRS, SELL])
def test_back_to_back_after_abort(hp, gpu, keep_sell, kernel):
    prob = hp.generate_matrix(*DIMS)
    b1, b2 = _rhs(prob)
    want2 = _fresh(hp, prob, kernel, b2, 60)
    M = hp.Matrix.from_hpc(prob)
    M.set_option("spmv_kernel", kernel)
    solve_bits(hp, M, b1, 60)
    M.set_option("spin_budget_us", 20000)
    M.set_option("dbg_withhold", 3)
    with pytest.raises(hp.HPCCGError, match="device wait timed out"):
        solve_bits(hp, M, b1, 60)
    M.set_option("dbg_withhold", 0)
    assert solve_bits(hp, M, b2, 60) == want2
    M.close()


def test_back_to_back_options(hp, gpu):
    """Option changes between solves (graph on/off, event timing, fused update
    off and on) leave the next default solve bitwise a fresh one."""
    prob = hp.generate_matrix(*DIMS)
    b1, b2 = _rhs(prob)
    want2 = _fresh(hp, prob, DIRECT, b2, 60)
    M = hp.Matrix.from_hpc(prob)
    M.set_option("spmv_kernel", DIRECT)
    for k, v in (("event_timing", 1), ("use_graph", 0), ("fuse_update", 0), ("x_defer", 1)):
        M.set_option(k, v)
        solve_bits(hp, M, b1, 45)
    for k, v in (("event_timing", 0), ("use_graph", 1), ("fuse_update", -1), ("x_defer", 2)):
        M.set_option(k, v)
    assert M.get_option("fuse_update") == 1
    assert solve_bits(hp, M, b2, 60) == want2
    M.close()


def test_back_to_back_group(hp, gpu):
    """An in-process group of two ranks: b1 then b2 on the same members is
    bitwise a fresh group's b2 solve."""
    import torch

    def run(Ms, bs):
        xs = [torch.zeros(M.info()["nrow"], dtype=torch.float64, device=gpu) for M in Ms]
        _, it, nr, _ = hp.group_HPCCG(Ms, bs, xs, max_iter=50, tolerance=0.0)
        return it, nr, Ms[0].last_trace().tobytes(), b"".join(x.cpu().numpy().tobytes() for x in xs)

    def rhs2(Ms):  # b2 = 0.5 b + 1 on the device (waxpby.cpp:69-93 through the kernel ABI)
        out = []
        for M in Ms:
            n = M.info()["nrow"]
            ones = torch.ones(n, dtype=torch.float64, device=gpu)
            b2 = torch.empty(n, dtype=torch.float64, device=gpu)
            hp.waxpby(n, 0.5, M.vectors()[0], 1.0, ones, b2)
            out.append(b2)
        return out

    F = hp.group_generate(24, 20, 18, 2)
    want2 = run(F, rhs2(F))
    for M in F:
        M.close()
    Ms = hp.group_generate(24, 20, 18, 2)
    run(Ms, [M.vectors()[0] for M in Ms])
    assert run(Ms, rhs2(Ms)) == want2
    for M in Ms:
        M.close()
