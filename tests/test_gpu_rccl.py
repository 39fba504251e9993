"""RCCL through the library on one GPU: bootstrap (ncclGetUniqueId /
ncclCommInitRank), an all-reduce on the library's stream and teardown, with a
1-rank communicator. Two ranks cannot share a GPU under RCCL ("Duplicate GPU
detected"), so the multi-rank kernels are covered by the in-process group
(test_gpu_group.py) and the RCCL transport's call pattern by the gloo
emulation (test_multirank_cpu.py)."""
import numpy as np
import pytest

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
