"""The placement probe (hpccg_hip_probe_placement):
moving the values image and the p ring to other physical memory changes no
result (bitwise), the probe records one time per candidate, keeps the fastest
values, then ring, r and Ap placement, and the creation-time probe follows hpccg_hip_set_placement_probe."""
import numpy as np
import pytest

from test_gpu_parity import DIRECT, PAIRS, solve_bits

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kernel", [PAIRS, DIRECT])
def test_probe_keeps_bits(hp, gpu, kernel):
    prob = hp.generate_matrix(40, 36, 30)
    M = hp.Matrix.from_hpc(prob)
    M.set_option("spmv_kernel", kernel)
    assert M.placement().size == 0  # small image: the automatic probe is off
    base = solve_bits(hp, M, prob.b, 40)
    us = M.probe_placement(3)
    assert us.shape == (13,) and np.all(us > 0)
    pick = M.get_option("placement_pick")
    best = us[0]
    for phase in range(4):  # values, ring, r, Ap: each keeps the fastest so far
        cand = us[1 + 3 * phase:4 + 3 * phase]
        want = int(np.argmin(cand)) + 1 if cand.min() < best else 0
        assert (pick >> (8 * phase)) & 255 == want, (phase, us, pick)
        best = min(best, cand.min())
    assert solve_bits(hp, M, prob.b, 40) == base
    import torch
    assert solve_bits(hp, M, torch.as_tensor(prob.b, device=gpu), 40, gpu=gpu) == base
    M.probe_placement(0)  # no-op
    assert M.placement().size == 0 and M.get_option("placement_pick") == 0
    assert solve_bits(hp, M, prob.b, 40) == base
    with pytest.raises(hp.HPCCGError):
        M.probe_placement(17)
    M.close()


def test_probe_at_creation(hp, gpu):
    prob = hp.generate_matrix(32, 32, 32)
    M0 = hp.Matrix.from_hpc(prob)
    base = solve_bits(hp, M0, prob.b, 30)
    M0.close()
    try:
        hp.set_placement_probe(2)
        M = hp.Matrix.from_hpc(prob)
        assert M.placement().shape == (9,), {k: M.get_option(k) for k in ("has_a", "a_reject", "spmv_kernel", "a_width")}
        assert solve_bits(hp, M, prob.b, 30) == base
        M.close()
        G = hp.Matrix.generate(32, 32, 32)
        assert G.placement().shape == (9,), {k: G.get_option(k) for k in ("has_a", "a_reject", "spmv_kernel", "a_width")}
        G.close()
        with pytest.raises(hp.HPCCGError):
            hp.set_placement_probe(-2)
    finally:
        hp.set_placement_probe(0)


def test_probe_group_members(hp, gpu):
    """Members with ghost planes are timed as one rank (no halo, no
    all-reduce); the group solve afterwards is unchanged bitwise."""
    import torch
    Ms = hp.group_generate(24, 20, 18, 3)
    assert all(M.placement().size == 0 for M in Ms)  # no automatic probe for members

    def run():
        xs = [torch.zeros(M.info()["nrow"], dtype=torch.float64, device=gpu) for M in Ms]
        _, it, nr, _ = hp.group_HPCCG(Ms, [M.vectors()[0] for M in Ms], xs, max_iter=40, tolerance=0.0)
        return it, nr, Ms[0].last_trace().tobytes(), b"".join(x.cpu().numpy().tobytes() for x in xs)

    base = run()
    for M in Ms:
        assert M.probe_placement(2).shape == (9,)
    assert run() == base
    for M in Ms:
        M.close()
