"""Group fold (always on where it applies; get_option("group_fold") reports
whether the last solve used it): an in-process group run in member order sums
its two dots in the last member's kernels -- the same rank-ordered sum
k_group_sum makes (ddot.cpp:79-80's MPI_Allreduce) -- instead of a
k_group_sum launch per dot. Bar: bitwise the k_finalize + k_group_sum group
(fold 0) on every kernel, graph and eager, halo by pull and by plane copies,
2 and 3 members; off where it does not apply (peer all-reduce, k_finalize)."""
import pytest

pytestmark = pytest.mark.gpu


def _solve(hp, gpu, dims, P, p7, opts, max_iter=60):
    import torch
    Ms = hp.group_generate(*dims, P, use_7pt=p7)
    for M in Ms:
        for k, v in opts.items():
            M.set_option(k, v)
    xs = [torch.zeros(M.info()["nrow"], dtype=torch.float64, device=gpu) for M in Ms]
    _, it, nr, _ = hp.group_HPCCG(Ms, [M.vectors()[0] for M in Ms], xs, max_iter=max_iter)
    got = (it, nr, Ms[0].last_trace().tobytes(), b"".join(x.cpu().numpy().tobytes() for x in xs))
    used = Ms[0].get_option("group_fold")
    for M in Ms:
        M.close()
    return got, used


CASES = {
    "direct_2": ((24, 20, 9), 2, False, {"spmv_kernel": 1}, 1),
    "direct_3": ((20, 18, 10), 3, False, {"spmv_kernel": 1}, 1),
    "pairs_2": ((24, 20, 9), 2, False, {"spmv_kernel": 2}, 1),
    "pairs_3": ((24, 20, 9), 3, False, {"spmv_kernel": 2}, 1),
    "7pt_2": ((20, 18, 16), 2, True, {}, 1),
    "eager_3": ((20, 18, 10), 3, False, {"use_graph": 0}, 1),
    "planes_2": ((24, 20, 9), 2, False, {"halo_pull": 0}, 1),
    "finalize_2": ((24, 20, 9), 2, False, {"fold": 0}, 0),
    "peer_2": ((24, 20, 9), 2, False, {"peer_allreduce": 1}, 0),
}


@pytest.mark.parametrize("case", list(CASES))
def test_group_fold_bitwise(hp, gpu, case):
    dims, P, p7, opts, want = CASES[case]
    ref, used0 = _solve(hp, gpu, dims, P, p7, dict(opts, fold=0))
    got, used1 = _solve(hp, gpu, dims, P, p7, opts)
    assert used0 == 0 and used1 == want
    assert got == ref


def test_group_fold_back_to_back(hp, gpu):
    """Two solves on one group, the second with another right-hand side, equal
    a fresh group's solve of it (the last member's table and fold state carry
    nothing between solves)."""
    import torch
    dims = (24, 20, 9)

    def run(Ms, scale):
        xs = [torch.zeros(M.info()["nrow"], dtype=torch.float64, device=gpu) for M in Ms]
        bs = [2.0 + scale * torch.sin(torch.arange(M.info()["nrow"], dtype=torch.float64, device=gpu) * 0.37)
              for M in Ms]
        _, it, nr, _ = hp.group_HPCCG(Ms, bs, xs, max_iter=50)
        return it, nr, b"".join(x.cpu().numpy().tobytes() for x in xs)

    Ms = hp.group_generate(*dims, 2)
    run(Ms, 1.0)
    second = run(Ms, 0.75)
    for M in Ms:
        M.close()
    Fs = hp.group_generate(*dims, 2)
    fresh = run(Fs, 0.75)
    for M in Fs:
        M.close()
    assert second == fresh
