"""Peer-memory all-reduce of the two CG scalars (option "peer_allreduce"; RCCL
stays the default): the lane that completes a local dot stores it into every
rank's mailbox and sums the ranks' values in rank order inside the kernel
(ddot.cpp:79-80's MPI_Allreduce without a collective call). On one GPU it
runs in an in-process group of two ranks (members launched eagerly on their
own streams: their kernels wait for each other) and in the 1-rank emulation of
the multi-rank iteration, where it also carries the update into the SpMV
launch. Bars: bitwise the default solve, whose scalars the group sums in rank
order (k_group_sum) -- the same order the kernels use."""
import time

import pytest

pytestmark = pytest.mark.gpu


def _group(hp, dims, p7, opts, peer, max_iter=80, withhold=0):
    import torch
    Ms = hp.group_generate(*dims, 2, use_7pt=p7)
    for M in Ms:
        for k, v in opts.items():
            M.set_option(k, v)
        M.set_option("peer_allreduce", peer)
    if withhold:
        Ms[1].set_option("spin_budget_us", 20000)
        Ms[1].set_option("dbg_withhold", withhold)
        Ms[0].set_option("spin_budget_us", 20000)
    n = dims[0] * dims[1] * dims[2]
    xs = [torch.zeros(n, dtype=torch.float64, device="cuda:0") for _ in Ms]
    bs = [M.vectors()[0] for M in Ms]
    _, it, nr, times = hp.group_HPCCG(Ms, bs, xs, max_iter=max_iter)
    assert Ms[0].get_option("peer_allreduce") == peer
    if peer:
        assert Ms[0].get_option("graph_used") == 0  # members side by side, never one graph
    return (it, nr, Ms[0].last_trace().tobytes(), [x.cpu().numpy().tobytes() for x in xs]), Ms, times


CASES = {
    "direct": ((24, 20, 9), False, {"spmv_kernel": 1}),
    "pairs": ((24, 20, 9), False, {"spmv_kernel": 2}),
    "direct_7pt": ((20, 18, 16), True, {}),
    "sell": ((16, 16, 12), False, {"spmv_kernel": 0}),
    "unfused": ((16, 16, 12), False, {"fuse_p": 0}),
    "finalize": ((16, 16, 12), False, {"fold": 0}),
}


@pytest.mark.parametrize("case", list(CASES))
def test_peer_allreduce_group_bitwise(hp, gpu, case):
    dims, p7, opts = CASES[case]
    if opts.get("spmv_kernel") == 0:
        hp.set_keep_sell(True)
    try:
        ref, _, _ = _group(hp, dims, p7, opts, 0)
        got, Ms, times = _group(hp, dims, p7, opts, 1)
    finally:
        hp.set_keep_sell(False)
    assert got == ref
    assert times[4] > 0.0  # the all-reduce class is stamped in the kernels


def test_peer_allreduce_emulated_fused_update(hp, gpu):
    """force_comm 2 (the multi-rank iteration on a 1-rank communicator) with the
    peer all-reduce: both scalars summed in the kernels, so the update runs
    inside the SpMV launch again (one launch per iteration plus the r planes'
    RCCL group). Bitwise the plain single-rank solve, graph and eager."""
    import torch
    hp.comm_init(hp.comm_unique_id(), 1, 0)
    try:
        M = hp.Matrix.generate(40, 36, 30)
        b, _, _ = M.vectors()
        outs = []
        for fc, peer, graph in ((0, 0, 1), (2, 0, 1), (2, 1, 1), (2, 1, 0)):
            M.set_option("force_comm", fc)
            M.set_option("peer_allreduce", peer)
            M.set_option("use_graph", graph)
            x = torch.zeros(40 * 36 * 30, dtype=torch.float64, device=gpu)
            _, it, nr, times = hp.HPCCG(M, b, x, max_iter=120, device=True)
            outs.append((it, nr, M.last_trace().tobytes(), x.cpu().numpy().tobytes()))
            assert M.get_option("fuse_update") == (1 if (fc == 0 or peer) else 0)
            if fc:  # (the plain single-rank solve is the persistent launch: no graph)
                assert M.get_option("graph_used") == graph
        for o in outs[1:]:
            assert o == outs[0]
        M.close()
    finally:
        hp.comm_destroy()


def test_peer_allreduce_wait_is_bounded(hp, gpu):
    """Member 1 withholds a p.Ap partial: its own slot wait gives up, and member
    0's wait for member 1's contribution must give up too -- an error, not a
    hang -- and the next group solve is bitwise the default one."""
    ref, _, _ = _group(hp, (16, 16, 12), False, {}, 0, max_iter=30)
    t0 = time.time()
    with pytest.raises(hp.HPCCGError, match="device wait timed out"):
        _group(hp, (16, 16, 12), False, {}, 1, max_iter=30, withhold=2)
    assert time.time() - t0 < 20.0
    got, _, _ = _group(hp, (16, 16, 12), False, {}, 1, max_iter=30)
    assert got == ref


def test_peer_allreduce_auto_default(hp, gpu):
    """Option peer_allreduce -1 (auto, the default): the multi-rank iteration
    of the 1-rank emulation sums its scalars in the kernels and runs the update
    inside the SpMV launch (one launch per iteration plus r's planes), while a
    single rank and an in-process group keep their own paths; bitwise the plain
    solve either way. (An RCCL job decides at creation from a collective
    self-test: tests/rccl_worker.py.)"""
    import torch
    hp.comm_init(hp.comm_unique_id(), 1, 0)
    try:
        M = hp.Matrix.generate(40, 36, 30)
        b, _, _ = M.vectors()
        assert M.get_option("peer_allreduce") == 0  # one rank: nothing to sum
        outs = []
        for fc in (0, 2):
            M.set_option("force_comm", fc)
            x = torch.zeros(40 * 36 * 30, dtype=torch.float64, device=gpu)
            _, it, nr, _ = hp.HPCCG(M, b, x, max_iter=120, device=True)
            outs.append((it, nr, M.last_trace().tobytes(), x.cpu().numpy().tobytes()))
            assert M.get_option("fuse_update") == 1
            assert M.get_option("peer_allreduce") == (1 if fc == 2 else 0)
        assert outs[0] == outs[1]
        M.close()
    finally:
        hp.comm_destroy()
    Ms = hp.group_generate(24, 20, 9, 2)
    assert all(m.get_option("peer_allreduce") == 0 for m in Ms)
    for m in Ms:
        m.close()
