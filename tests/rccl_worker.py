"""One rank of the 2-process RCCL test (tests/test_gpu_rccl.py): gloo carries
the unique id, RCCL the data path. Checks the 27pt_8x8x8_x2ranks golden."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from conftest import (RTRANS_RTOL_MULTI, check_final, check_trace, load_pkg, solve_case,  # noqa: E402
                      unhex)


def main():
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    hp = load_pkg()
    torch.cuda.set_device(local)
    hp.set_device(local)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    obj = [hp.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    hp.comm_init(obj[0], world, rank)
    with open(os.path.join(HERE, "golden", "golden.json")) as f:
        c = solve_case(json.load(f), "27pt_8x8x8_x2ranks")
    assert c["ranks"] == world
    M = hp.Matrix.generate(c["nx"], c["ny"], c["nz"])
    b, _, _ = M.vectors()
    n = c["nx"] * c["ny"] * c["nz"]
    x = torch.zeros(n, dtype=torch.float64, device=f"cuda:{local}")
    auto = M.get_option("peer_allreduce")  # the creation-time self-test's verdict (auto mode)
    M.set_option("peer_allreduce", 0)  # first the scalars through RCCL
    _, it, nr, times = hp.HPCCG(M, b, x, max_iter=500, device=True)
    tr = M.last_trace()
    ref_tr = [unhex(t) for t in c["trace_normr"]]
    rr = c["runs"]["500"]
    assert tr[0] == ref_tr[0]
    assert check_trace(tr, ref_tr, RTRANS_RTOL_MULTI) >= 5
    check_final(it, nr, tr, rr["niters"], unhex(rr["normr"]), ref_tr, 500)
    assert (x - 1.0).abs().max().item() <= 1e-12
    assert times[4] > 0.0 and times[5] > 0.0
    # the peer-memory all-reduce (IPC-mapped mailboxes, summed in the kernels,
    # the update fused into the SpMV launch): two ranks, so the rank-order sum
    # is RCCL's sum bit for bit -- the whole solve must be
    got = (it, nr, tr.tobytes(), x.cpu().numpy().tobytes())
    assert auto == 1, "the peer all-reduce self-test failed on two GPUs"
    M.set_option("peer_allreduce", -1)  # the default
    x.zero_()
    _, it2, nr2, _ = hp.HPCCG(M, b, x, max_iter=500, device=True)
    assert M.get_option("peer_allreduce") == 1 and M.get_option("fuse_update") == (1 if M.get_option("spmv_kernel") == 1 else 0)
    assert (it2, nr2, M.last_trace().tobytes(), x.cpu().numpy().tobytes()) == got
    # the default pulls in-launch (halo_pull 2: the neighbours' r read by the
    # fused launch's ghost blocks, or the update's trailing blocks, after r.r);
    # k_pull before the SpMV launch (halo_pull 1) gives the same bits
    pull_auto = M.get_option("halo_pull")
    assert pull_auto in (0, 2)
    M.set_option("halo_pull", 1)
    x.zero_()
    _, it3, nr3, _ = hp.HPCCG(M, b, x, max_iter=500, device=True)
    assert M.get_option("halo_pull") == (1 if pull_auto else 0)
    assert (it3, nr3, M.last_trace().tobytes(), x.cpu().numpy().tobytes()) == got
    graph_used = M.get_option("graph_used")
    M.close()
    # the collective fallback: rank 1's production-protocol
    # self-test fails (HPCCG_DBG_FAIL_PROTO) -- every rank must reach the same
    # verdict (both in-kernel transports off) and solve through RCCL: the
    # scalars by ncclAllReduce, r's planes by ncclSend/ncclRecv
    if rank == 1:
        os.environ["HPCCG_DBG_FAIL_PROTO"] = "1"
    F = hp.Matrix.generate(c["nx"], c["ny"], c["nz"])
    os.environ.pop("HPCCG_DBG_FAIL_PROTO", None)
    verdicts = [F.get_option(k) for k in ("peer_auto_ok", "pull_auto_ok", "proto_auto_ok")]
    assert verdicts == [0, 0, 0], verdicts
    assert F.get_option("peer_allreduce") == 0 and F.get_option("halo_pull") == 0
    b, _, _ = F.vectors()
    x.zero_()
    _, it4, nr4, times4 = hp.HPCCG(F, b, x, max_iter=500, device=True)
    assert (it4, nr4, F.last_trace().tobytes(), x.cpu().numpy().tobytes()) == got
    assert times4[4] > 0.0 and times4[5] > 0.0  # (RCCL's all-reduce and plane exchange stamped)
    F.close()
    print(f"RCCL-WORKER-OK rank {rank} graph_used={graph_used}", flush=True)
    hp.comm_destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
