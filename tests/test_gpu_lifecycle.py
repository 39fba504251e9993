"""Matrix lifecycle: creating, solving and destroying matrices again and again
returns every device byte (the image, the p ring, the persistent launch's dot
slots, the graph, the event pool, the pinned readback buffer), through each
entry point -- device generator, host struct, CSR, the drop-in cache and the
in-process group. A long-running caller (a service solving many systems)
would otherwise run the HBM out; HPCCG.cpp:396-398 frees its work vectors on
every call."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_bytes():
    import torch
    torch.cuda.synchronize()
    return torch.cuda.mem_get_info()[0]


def _cycle(hp, gpu, make, solves=2):
    import torch
    M = make()
    n = M.info()["nrow"]
    x = torch.zeros(n, dtype=torch.float64, device=gpu)
    b, _, _ = M.vectors()
    for _ in range(solves):
        x.zero_()
        hp.HPCCG(M, b, x, max_iter=30, device=True)
    M.set_option("event_timing", 1)  # the event pool too
    x.zero_()
    hp.HPCCG(M, b, x, max_iter=30, device=True)
    M.close()
    del x


@pytest.mark.parametrize("dims", [(64, 64, 64), (100, 100, 100), (40, 36, 30)])
def test_generate_solve_destroy_returns_memory(hp, gpu, dims):
    _cycle(hp, gpu, lambda: hp.Matrix.generate(*dims))  # warm: runtime pools, code objects
    before = _free_bytes()
    for _ in range(12):
        _cycle(hp, gpu, lambda: hp.Matrix.generate(*dims))
    after = _free_bytes()
    # 12 images of >= 18 MB each: a leak of any per-matrix buffer shows; allow
    # the runtime's own pool granularity
    assert before - after <= 64 << 20, (dims, (before - after) / 2**20)


def test_host_and_csr_entry_points_return_memory(hp, gpu):
    prob = hp.generate_matrix(48, 40, 36)
    rp, cols, vals = prob.to_csr()
    mk = [lambda: hp.Matrix.from_hpc(prob), lambda: hp.Matrix.from_csr(rp, cols, vals)]
    for f in mk:
        M = f()
        M.close()
    before = _free_bytes()
    for _ in range(8):
        for f in mk:
            M = f()
            x = np.zeros(M.info()["nrow"])
            hp.HPCCG(M, prob.b, x, max_iter=20)
            M.close()
    assert before - _free_bytes() <= 64 << 20
    prob.close()


def test_dropin_cache_release_returns_memory(hp, gpu):
    def once():
        prob = hp.generate_matrix(50, 50, 50)
        x = prob.x
        hp.dropin_HPCCG(prob, x, max_iter=20)
        hp.dropin_HPCCG(prob, prob.x, max_iter=20)  # the cached image
        assert hp.lib().hpccg_hip_dropin_cached(prob.A) == 1
        prob.close()  # destroyMatrix releases the cached image

    once()
    before = _free_bytes()
    for _ in range(8):
        once()
    assert before - _free_bytes() <= 64 << 20


def test_group_returns_memory(hp, gpu):
    import torch

    def once():
        Ms = hp.group_generate(32, 32, 16, 3)
        xs = [torch.zeros(M.info()["nrow"], dtype=torch.float64, device=gpu) for M in Ms]
        hp.group_HPCCG(Ms, [M.vectors()[0] for M in Ms], xs, max_iter=30)
        for M in Ms:
            M.close()

    once()
    before = _free_bytes()
    for _ in range(8):
        once()
    assert before - _free_bytes() <= 64 << 20
