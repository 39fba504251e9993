"""The host-bootstrapped communicator's plumbing on CPU (gloo, world_size 2 and
3): hpccg_hip_comm_init_host with torch.distributed's all-gather as the
callback, the mode it reports, and the host-value all-reduce that the CLI and
bench use for the reference's timing statistics (main.cpp:206-208) and
compute_residual's max (compute_residual.cpp:73), reduced in rank order
through the callback -- no GPU, no RCCL. The device side of the same
transport runs in tests/test_gpu_hostcomm.py."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from conftest import load_pkg


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# scenario -> (this rank's local {peer, pull, protocol} results, the job's verdict)
SCENARIOS = [
    (lambda r, w: (1, 1, 1), [1, 1, 1]),                          # every rank passed
    (lambda r, w: (1, 1, 0 if r == w - 1 else 1), [0, 0, 0]),     # the last rank's protocol test failed: both off
    (lambda r, w: (0 if r == 0 else 1, 1, 1), [0, 1, 0]),         # rank 0's peer test failed: the pull stays
    (lambda r, w: (1, 0 if r == 1 else 1, 1), [1, 0, 0]),         # rank 1's pull test failed: the peer stays
    (lambda r, w: (0 if r == 1 else 1, 1, 0 if r == 0 else 1), [0, 1, 0]),  # protocol counts only with both
]


def _local(sc, rank, world):
    return SCENARIOS[sc][0](rank, world)


def _worker(rank, world, port, q):
    import ctypes as C

    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {"rank": rank}
    try:
        hp = load_pkg()
        out["mode0"] = hp.comm_mode()
        hp.comm_init_host(world, rank)
        out["mode"] = hp.comm_mode()
        n, r = C.c_int(0), C.c_int(-1)
        hp.lib().hpccg_hip_comm_size(C.byref(n), C.byref(r))
        out["size"] = (n.value, r.value)
        v = np.array([0.1 * (rank + 1), -float(rank), 2.0 ** rank])
        out["sum"] = hp.comm_allreduce_host(v, "sum").tolist()
        out["min"] = hp.comm_allreduce_host(v, "min").tolist()
        out["max"] = hp.comm_allreduce_host(v, "max").tolist()
        # the self-tests' collective verdict: ranks with
        # different local results all reach the job's one verdict
        out["verdicts"] = [hp.transport_verdict(_local(sc, rank, world)) for sc in range(len(SCENARIOS))]
        hp.comm_destroy()
        out["mode_after"] = hp.comm_mode()
        # a callback that returns the wrong shape is refused at init (the
        # library checks that every rank sees every rank in order)
        try:
            hp.comm_init_host(world, rank, allgather=lambda data: [data] * (world + 1))
            out["bad_cb"] = "accepted"
        except hp.HPCCGError as e:
            out["bad_cb"] = str(e)
        out["mode_bad"] = hp.comm_mode()
    except Exception as e:  # reported to the test
        out["error"] = repr(e)
    finally:
        q.put(out)
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_host_bootstrap_allreduce(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    outs = sorted([q.get(timeout=240) for _ in range(world)], key=lambda d: d["rank"])
    for p in ps:
        p.join(timeout=60)
    vs = [np.array([0.1 * (r + 1), -float(r), 2.0 ** r]) for r in range(world)]
    want_sum = np.zeros(3)
    for v in vs:  # rank order from 0.0, as the library adds them
        want_sum = want_sum + v
    for d in outs:
        assert "error" not in d, d
        assert d["mode0"] == "none" and d["mode"] == "host" and d["mode_after"] == "none"
        assert d["size"] == (world, d["rank"])
        assert np.array(d["sum"]).tobytes() == want_sum.tobytes()
        assert d["min"] == np.min(vs, axis=0).tolist() and d["max"] == np.max(vs, axis=0).tolist()
        assert "comm_init_host failed" in d["bad_cb"] and d["mode_bad"] == "none"
        assert d["verdicts"] == [want for _, want in SCENARIOS], d["verdicts"]
