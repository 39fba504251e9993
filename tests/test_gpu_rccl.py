"""RCCL through the library: bootstrap (ncclGetUniqueId / ncclCommInitRank),
an all-reduce on the library's stream and teardown with a 1-rank
communicator; the CG's two scalars routed through ncclAllReduce inside the
captured hipGraph (force_comm, 1 rank); and, where two GPUs are visible, the
real 2-process RCCL job (one rank per GPU, halo by ncclSend/Recv, scalars by
ncclAllReduce) against the reference's 2-rank golden. Two ranks cannot share
a GPU under RCCL ("Duplicate GPU detected"), so on a 1-GPU box the multi-rank
kernels are covered by the in-process group (test_gpu_group.py) and the RCCL
call pattern by the gloo emulation (test_multirank_cpu.py)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_rccl_one_rank_comm(hp, gpu):
    uid = hp.comm_unique_id()
    assert len(uid) == 128
    hp.comm_init(uid, 1, 0)
    try:
        v = np.array([1.5, -2.0, 3.25])
        for op in ("sum", "min", "max"):
            assert np.array_equal(hp.comm_allreduce_host(v, op), v)
        # a solve with the communicator up still takes the single-rank path
        M = hp.Matrix.generate(12, 12, 12)
        import torch
        b, _, _ = M.vectors()
        x = torch.zeros(12 ** 3, dtype=torch.float64, device=gpu)
        _, it, nr, times = hp.HPCCG(M, b, x, max_iter=60, device=True)
        assert it == 59 and times[4] == 0.0 and times[5] == 0.0
        M.close()
    finally:
        hp.comm_destroy()


@pytest.mark.parametrize("graph", [1, 0])
def test_rccl_scalars_in_graph(hp, gpu, graph):
    """force_comm: p.Ap and r.r go loc -> ncclAllReduce -> g, as on several
    ranks, with the RCCL calls captured into the CG hipGraph; a 1-rank sum is
    the identity, so the solve is bitwise the plain one."""
    import torch
    hp.comm_init(hp.comm_unique_id(), 1, 0)
    try:
        M = hp.Matrix.generate(40, 36, 30)
        b, _, _ = M.vectors()
        outs = []
        for fc in (0, 1):
            M.set_option("force_comm", fc)
            M.set_option("use_graph", graph)
            x = torch.zeros(40 * 36 * 30, dtype=torch.float64, device=gpu)
            _, it, nr, times = hp.HPCCG(M, b, x, max_iter=120, device=True)
            outs.append((it, nr, M.last_trace().tobytes(), x.cpu().numpy().tobytes()))
            if fc:
                assert times[4] > 0.0  # the all-reduce class was stamped
                assert M.get_option("graph_used") == graph
        assert outs[0] == outs[1]
        M.close()
    finally:
        hp.comm_destroy()


def test_rccl_emulated_multirank_iteration(hp, gpu):
    """force_comm 2 on a 1-rank communicator: the multi-rank iteration shape
    (k_p_boundary path, the halo as a plane-sized ncclSend/ncclRecv to itself,
    both scalars through ncclAllReduce) in a captured hipGraph and eagerly,
    halo in line and (eager) on the second stream. Every variant is bitwise the
    plain solve. This is the capture the N > 1 RCCL job replays: with the halo
    on a forked stream it segfaulted inside the ROCm runtime, so graphs run it
    in line."""
    import torch
    hp.comm_init(hp.comm_unique_id(), 1, 0)
    try:
        M = hp.Matrix.generate(40, 36, 30)
        b, _, _ = M.vectors()
        outs = []
        for fc, graph in ((0, 1), (2, 1), (2, 0)):
            M.set_option("force_comm", fc)
            M.set_option("use_graph", graph)
            x = torch.zeros(40 * 36 * 30, dtype=torch.float64, device=gpu)
            _, it, nr, times = hp.HPCCG(M, b, x, max_iter=120, device=True)
            outs.append((it, nr, M.last_trace().tobytes(), x.cpu().numpy().tobytes()))
            if fc:  # (the plain single-rank solve is the persistent launch: no graph)
                assert M.get_option("graph_used") == graph
            if fc:
                assert times[4] > 0.0
        for o in outs[1:]:
            assert o == outs[0]
        M.close()
    finally:
        hp.comm_destroy()


def test_rccl_two_processes(hp, gpu, golden):
    """The RCCL job itself: torch.distributed.run launches 2 ranks, one per
    GPU; each generates its z-slab of the 2 x 8^3 problem on its GPU and
    solves with the RCCL halo + all-reduce, graph-replayed; the trace must
    meet the reference's 2-rank golden (27pt_8x8x8_x2ranks, 1e-7). Then the
    in-kernel transport (peer all-reduce, in-launch pull) bitwise, and the
    collective fallback: rank 1's protocol self-test fails on purpose
    (HPCCG_DBG_FAIL_PROTO), both ranks turn the in-kernel transport off and
    the RCCL solve gives the same bits."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two visible GPUs (RCCL refuses two ranks on one GPU)")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", "29517",
                        os.path.join(ROOT, "tests", "rccl_worker.py")],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "RCCL-WORKER-OK rank 0" in r.stdout and "RCCL-WORKER-OK rank 1" in r.stdout
