"""The r-halo by pull (option halo_pull, on by default where it applies): each
rank's ghost planes of r are read from its neighbours' boundary rows right
before its SpMV launch (exchange_externals.cpp:87-126 moves the same values
by MPI), instead of a send/recv group after the update. On one GPU it runs in
the in-process group (the members' buffers) and in the 1-rank emulation (its
own rows into scratch); an RCCL job maps its neighbours' r through IPC after a
collective test (tests/rccl_worker.py). halo_pull 2 pulls inside the
iteration's last launch once its r.r completion is in (with the peer
all-reduce; the default there, else k_pull):
the fused launch's ghost blocks, or trailing blocks of the update. Bars:
bitwise the plane-copy halo, on every kernel, graph and eager, with RCCL-style
and peer all-reduces; the fused update in a group (fuse_update 2, members small
enough to be resident side by side) bitwise the unfused group."""
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
    fu = Ms[0].get_option("fuse_update")
    for M in Ms:
        M.close()
    return got, pull, fu


# name: dims, ranks, 7-pt, options, the halo_pull in effect with those options
CASES = {
    "direct_2": ((24, 20, 9), 2, False, {"spmv_kernel": 1}, 1),
    "direct_3": ((20, 18, 10), 3, False, {"spmv_kernel": 1}, 1),
    "pairs_2": ((24, 20, 9), 2, False, {"spmv_kernel": 2}, 1),
    "pairs_3": ((20, 18, 10), 3, False, {"spmv_kernel": 2}, 1),
    "7pt_2": ((20, 18, 16), 2, True, {}, 1),
    "eager_3": ((20, 18, 10), 3, False, {"use_graph": 0}, 1),
    # with the peer all-reduce the default pulls in-launch
    "peer_2": ((24, 20, 9), 2, False, {"peer_allreduce": 1}, 2),
    "peer_pairs_2": ((24, 20, 9), 2, False, {"peer_allreduce": 1, "spmv_kernel": 2}, 2),
    "peer_kpull_2": ((24, 20, 9), 2, False, {"peer_allreduce": 1, "halo_pull": 1}, 1),
    # in-launch: trailing pull blocks of k_update (and of the prologue's)
    "inlaunch_direct_2": ((24, 20, 9), 2, False, {"peer_allreduce": 1, "spmv_kernel": 1, "halo_pull": 2}, 2),
    "inlaunch_pairs_2": ((24, 20, 9), 2, False, {"peer_allreduce": 1, "spmv_kernel": 2, "halo_pull": 2}, 2),
    # without the peer all-reduce the in-launch request falls back to k_pull
    "inlaunch_no_peer_2": ((24, 20, 9), 2, False, {"spmv_kernel": 1, "halo_pull": 2}, 1),
    # the fused update in a group: the ghost / pull blocks after the update
    # blocks; a 4096-row ghost plane takes several ghost blocks
    "fused_kpull_2": ((64, 64, 4), 2, False,
                      {"peer_allreduce": 1, "spmv_kernel": 1, "fuse_update": 2, "halo_pull": 1}, 1),
    "fused_inlaunch_2": ((64, 64, 4), 2, False, {"peer_allreduce": 1, "spmv_kernel": 1, "fuse_update": 2}, 2),
    "fused_7pt_inlaunch_2": ((64, 48, 6), 2, True,
                             {"peer_allreduce": 1, "spmv_kernel": 1, "fuse_update": 2, "halo_pull": 2}, 2),
}


@pytest.mark.parametrize("case", list(CASES))
def test_pull_group_bitwise(hp, gpu, case):
    dims, P, p7, opts, want = CASES[case]
    ref, pull0, _ = _group_solve(hp, gpu, dims, P, p7, dict(opts, halo_pull=0))
    got, pull1, fu = _group_solve(hp, gpu, dims, P, p7, opts)
    assert pull0 == 0 and pull1 == want
    assert fu == (1 if opts.get("fuse_update") == 2 else fu)
    assert got == ref


@pytest.mark.parametrize("p7", [False, True])
def test_fused_group_equals_unfused(hp, gpu, p7):
    """The fused launch's ghost blocks (after its update blocks) store every
    ghost row of p_k: the fused group with the in-launch pull is bitwise the
    default (unfused, RCCL-style sums, k_pull) group."""
    dims = (64, 64, 4) if not p7 else (64, 48, 6)
    ref, _, fu0 = _group_solve(hp, gpu, dims, 2, p7, {"spmv_kernel": 1})
    got, pull, fu1 = _group_solve(hp, gpu, dims, 2, p7,
                                  {"spmv_kernel": 1, "peer_allreduce": 1, "fuse_update": 2, "halo_pull": 2})
    assert fu0 == 0 and fu1 == 1 and pull == 2
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
        for fc, peer, pull, graph in ((0, -1, -1, 1), (2, -1, -1, 1), (2, 0, -1, 1), (2, -1, -1, 0), (2, 0, 0, 1),
                                      (2, -1, 1, 1), (2, -1, 1, 0), (2, 0, 2, 1)):
            M.set_option("force_comm", fc)
            M.set_option("peer_allreduce", peer)
            M.set_option("halo_pull", pull)
            M.set_option("use_graph", graph)
            x = torch.zeros(40 * 36 * 30, dtype=torch.float64, device=gpu)
            _, it, nr, times = hp.HPCCG(M, b, x, max_iter=120, device=True)
            outs.append((it, nr, M.last_trace().tobytes(), x.cpu().numpy().tobytes()))
            want = 0 if fc != 2 or pull == 0 else (2 if pull != 1 and peer != 0 else 1)
            assert M.get_option("halo_pull") == want
            if fc == 2 and pull != 0:
                assert times[5] > 0.0  # the halo class is stamped by the pull
        for o in outs[1:]:
            assert o == outs[0]
        M.close()
    finally:
        hp.comm_destroy()
