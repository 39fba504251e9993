"""The r-halo by pull (option halo_pull, on by default where it applies): each
rank's ghost planes of r are read from its neighbours' boundary rows right
before its SpMV launch (exchange_externals.cpp:87-126 moves the same values
by MPI), instead of a send/recv group after the update. On one GPU it runs in
the in-process group (the members' buffers) and in the 1-rank emulation (its
own rows into scratch); an RCCL job maps its neighbours' r through IPC after a
collective test (tests/rccl_worker.py). Bars: bitwise the plane-copy halo, on
every kernel, graph and eager, with RCCL-style and peer all-reduces."""
import pytest

pytestmark = pytest.mark.gpu


def _group_solve(hp, gpu, dims, P, p7, opts, max_iter=60):
    import torch
    Ms = hp.group_generate(*dims, P, use_7pt=p7)
    for M in Ms:
        for k, v in opts.items():
            M.set_option(k, v)
    xs = [torch.zeros(M.info()["nrow"], dtype=torch.float64, device=gpu) for M in Ms]
    _, it, nr, _ = hp.group_HPCCG(Ms, [M.vectors()[0] for M in Ms], xs, max_iter=max_iter)
    got = (it, nr, Ms[0].last_trace().tobytes(), b"".join(x.cpu().numpy().tobytes() for x in xs))
    pull = Ms[0].get_option("halo_pull")
    for M in Ms:
        M.close()
    return got, pull


CASES = {
    "direct_2": ((24, 20, 9), 2, False, {"spmv_kernel": 1}),
    "direct_3": ((20, 18, 10), 3, False, {"spmv_kernel": 1}),
    "pairs_2": ((24, 20, 9), 2, False, {"spmv_kernel": 2}),
    "pairs_3": ((20, 18, 10), 3, False, {"spmv_kernel": 2}),
    "7pt_2": ((20, 18, 16), 2, True, {}),
    "eager_3": ((20, 18, 10), 3, False, {"use_graph": 0}),
    "peer_2": ((24, 20, 9), 2, False, {"peer_allreduce": 1}),
    "peer_pairs_2": ((24, 20, 9), 2, False, {"peer_allreduce": 1, "spmv_kernel": 2}),
}


@pytest.mark.parametrize("case", list(CASES))
def test_pull_group_bitwise(hp, gpu, case):
    dims, P, p7, opts = CASES[case]
    ref, pull0 = _group_solve(hp, gpu, dims, P, p7, dict(opts, halo_pull=0))
    got, pull1 = _group_solve(hp, gpu, dims, P, p7, opts)  # the default
    assert pull0 == 0 and pull1 == 1
    assert got == ref


def test_pull_emulated(hp, gpu):
    """force_comm 2 (the multi-rank iteration on a 1-rank communicator): the
    pull of an interior rank's two planes (into scratch) with RCCL and with
    peer all-reduces, graph and eager; bitwise the plain single-rank solve."""
    import torch
    hp.comm_init(hp.comm_unique_id(), 1, 0)
    try:
        M = hp.Matrix.generate(40, 36, 30)
        b, _, _ = M.vectors()
        outs = []
        for fc, peer, pull, graph in ((0, -1, -1, 1), (2, -1, -1, 1), (2, 0, -1, 1), (2, -1, -1, 0), (2, 0, 0, 1)):
            M.set_option("force_comm", fc)
            M.set_option("peer_allreduce", peer)
            M.set_option("halo_pull", pull)
            M.set_option("use_graph", graph)
            x = torch.zeros(40 * 36 * 30, dtype=torch.float64, device=gpu)
            _, it, nr, times = hp.HPCCG(M, b, x, max_iter=120, device=True)
            outs.append((it, nr, M.last_trace().tobytes(), x.cpu().numpy().tobytes()))
            assert M.get_option("halo_pull") == (1 if fc == 2 and pull != 0 else 0)
            if fc == 2 and pull != 0:
                assert times[5] > 0.0  # the halo class is stamped by the pull
        for o in outs[1:]:
            assert o == outs[0]
        M.close()
    finally:
        hp.comm_destroy()
