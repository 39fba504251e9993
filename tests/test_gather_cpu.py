"""The gather halo plan on the CPU (make_local_matrix.cpp:58-610,
exchange_externals.cpp:51-131).

* hpccg_gather_plan numbers the external columns exactly as the reference's
  make_local_matrix does (restated below in Python, line-for-line in
  behaviour: first appearance, owner = last rank whose start_row <= column,
  local indices assigned owner group by owner group);
* gloo, world_size 3 and 4: each rank reads its block of the Mode-2 system
  (read_HPC_row), takes the library's plan, sends its requests to the owners
  (the all-gathered P x P count matrix + one message per pair: the protocol
  rccl_requests runs over RCCL), then runs the CG recurrence with the halo
  moved by those send lists. The trace must match the serial reference trace
  of the same file (golden file_general_600) within the multi-rank tolerance.
"""
import math
import os
import socket
import sys

import numpy as np
import pytest

from conftest import RTRANS_RTOL_MULTI, ROOT, check_final, check_trace, load_pkg, solve_case, unhex

sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import filemode  # noqa: E402


def reference_externals(rp, cols, start, nrow, starts):
    """make_local_matrix.cpp:96-200 restated: (external_index in local order,
    owner per local external)."""
    externals = {}
    external_index = []
    for i in range(nrow):
        for e in range(rp[i], rp[i + 1]):
            c = int(cols[e])
            if start <= c < start + nrow:
                continue
            if c not in externals:
                externals[c] = len(external_index)
                external_index.append(c)
    size = len(starts)
    proc = []
    for c in external_index:
        for j in range(size - 1, -1, -1):
            if starts[j] <= c:
                proc.append(j)
                break
    local = [-1] * len(external_index)
    count = nrow
    for i in range(len(external_index)):
        if local[i] == -1:
            local[i] = count
            count += 1
            for j in range(i + 1, len(external_index)):
                if proc[j] == proc[i]:
                    local[j] = count
                    count += 1
    order = [None] * len(external_index)
    owner = [None] * len(external_index)
    for i, c in enumerate(external_index):
        order[local[i] - nrow] = c
        owner[local[i] - nrow] = proc[i]
    return order, owner


@pytest.fixture(scope="module")
def system_file(tmp_path_factory):
    rp, cl, vl, x0, b, xe = filemode.general_system(600)
    path = str(tmp_path_factory.mktemp("gather") / "general_600.dat")
    filemode.write(path, rp, cl, vl, x0, b, xe)
    return path


def _info(hp, probs):
    info = []
    for p in probs:
        rp, cols, _ = p.to_csr()
        h = hp.halo_plan(rp, cols, p.start_row, p.total_nrow)
        info += [p.nrow, h["ghost_lo"], h["ghost_hi"], p.start_row]
    return info


@pytest.mark.parametrize("P", [2, 3, 4, 7])
def test_gather_plan_matches_make_local_matrix(hp, system_file, P):
    probs = [hp.read_HPC_row(system_file, r, P) for r in range(P)]
    info = _info(hp, probs)
    starts = [p.start_row for p in probs]
    for p in probs:
        rp, cols, _ = p.to_csr()
        plan = hp.gather_plan(P, info, rp, cols, p.start_row)
        order, owner = reference_externals(rp, cols, p.start_row, p.nrow, starts)
        assert plan["ext_global"].tolist() == order
        runs = []
        for q in owner:
            if not runs or runs[-1][0] != q:
                runs.append([q, 0])
            runs[-1][1] += 1
        off = np.cumsum([0] + [c for _, c in runs])[:-1]
        assert plan["recv"] == [(q, int(o), c) for (q, c), o in zip(runs, off)]


def test_gather_plan_slab_problem(hp):
    """On the z-slab stencil the externals are the neighbour planes, in first
    appearance order (not sorted): the reference numbering, not the slab one."""
    P, nx, ny, nz = 3, 5, 4, 3
    probs = [hp.generate_matrix(nx, ny, nz, rank=r, size=P) for r in range(P)]
    info = []
    for r, p in enumerate(probs):
        rp, cols, _ = p.to_csr()
        h = hp.halo_plan(rp, cols, r * nx * ny * nz, P * nx * ny * nz)
        info += [nx * ny * nz, h["ghost_lo"], h["ghost_hi"], r * nx * ny * nz]
    starts = [r * nx * ny * nz for r in range(P)]
    rp, cols, _ = probs[1].to_csr()
    plan = hp.gather_plan(P, info, rp, cols, starts[1])
    order, _ = reference_externals(rp, cols, starts[1], nx * ny * nz, starts)
    assert plan["ext_global"].tolist() == order
    assert sorted(order) == list(range(starts[1] - nx * ny, starts[1])) + \
        list(range(starts[2], starts[2] + nx * ny))
    assert [q for q, _, _ in plan["recv"]] == [0, 2]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, path, max_iter, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hp = load_pkg()
        p = hp.read_HPC_row(path, rank, world)
        n, start = p.nrow, p.start_row
        rp, cols, vals = p.to_csr()
        h = hp.halo_plan(rp, cols, start, p.total_nrow)
        mine = torch.tensor([n, h["ghost_lo"], h["ghost_hi"], start], dtype=torch.int32)
        g = [torch.zeros(4, dtype=torch.int32) for _ in range(world)]
        dist.all_gather(g, mine)
        info = torch.cat(g).numpy()
        plan = hp.gather_plan(world, info, rp, cols, start)
        ext = plan["ext_global"]
        # requests to each owner, in our local order (rccl_requests over gloo)
        req = {qq: ext[o:o + c] for qq, o, c in plan["recv"]}
        counts = torch.tensor([len(req.get(qq, [])) for qq in range(world)], dtype=torch.int32)
        allc = [torch.zeros(world, dtype=torch.int32) for _ in range(world)]
        dist.all_gather(allc, counts)
        cnt = torch.stack(allc).numpy()  # cnt[q, r]: how many q requests from r
        ops, got = [], {}
        for qq in range(world):
            if cnt[rank, qq]:
                ops.append(dist.isend(torch.from_numpy(req[qq].astype(np.int64)), qq))
            if cnt[qq, rank]:
                got[qq] = torch.zeros(int(cnt[qq, rank]), dtype=torch.int64)
                ops.append(dist.irecv(got[qq], qq))
        for o in ops:
            o.wait()
        sends = {qq: got[qq].numpy() - start for qq in sorted(got)}  # local rows to pack
        # local CSR with own -> c - start, external -> n + j
        pos = {int(c): n + j for j, c in enumerate(ext)}
        lcols = np.array([c - start if start <= c < start + n else pos[int(c)] for c in cols], np.int64)
        pext = np.zeros(n + len(ext))

        def halo():
            ops, bufs = [], {}
            for qq, idx in sends.items():
                ops.append(dist.isend(torch.from_numpy(pext[idx].copy()), qq))
            for qq, o, c in plan["recv"]:
                bufs[qq] = (o, torch.zeros(c, dtype=torch.float64))
                ops.append(dist.irecv(bufs[qq][1], qq))
            for o in ops:
                o.wait()
            for qq, (o, t) in bufs.items():
                pext[n + o:n + o + len(t)] = t.numpy()

        def spmv():
            y = np.zeros(n)
            for i in range(n):
                s = 0.0
                for e in range(rp[i], rp[i + 1]):
                    s = s + vals[e] * pext[lcols[e]]
                y[i] = s
            return y

        def allsum(v):
            t = torch.tensor([v], dtype=torch.float64)
            dist.all_reduce(t)
            return t.item()

        b, x = p.b, p.x
        pext[:n] = x + 0.0 * x
        halo()
        r = b + (-1.0) * spmv()
        rr = allsum(float(np.dot(r, r)))
        hist, trace, niters = {}, [math.sqrt(rr)], 0
        for k in range(1, max_iter):
            chk = rr if k == 1 else hist[k - 2]
            if not math.sqrt(chk) > 0.0:
                break
            pext[:n] = r + 0.0 * r if k == 1 else r + (rr / hist[k - 2]) * pext[:n]
            hist[k - 1] = rr
            halo()
            Ap = spmv()
            alpha = rr / allsum(float(np.dot(pext[:n], Ap)))
            x = x + alpha * pext[:n]
            r = r + (-alpha) * Ap
            rr = allsum(float(np.dot(r, r)))
            niters = k
            trace.append(math.sqrt(hist[k - 1]))
        q.put((rank, niters, trace, float(np.max(np.abs(x - p.xexact))), len(ext)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [3, 4])
def test_gather_plan_cg_over_gloo(golden, system_file, world):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    max_iter = 120
    ps = [ctx.Process(target=_worker, args=(r, world, port, system_file, max_iter, q)) for r in range(world)]
    for pr in ps:
        pr.start()
    out = sorted(q.get(timeout=300) for _ in range(world))
    for pr in ps:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    c = solve_case(golden, "file_general_600")
    ref_tr = [unhex(t) for t in c["trace_normr"]]
    for rank, niters, trace, xerr, ne in out:
        assert trace == out[0][2]
        assert ne > 0
        assert trace[0] == ref_tr[0]
        assert check_trace(trace, ref_tr, RTRANS_RTOL_MULTI) >= 10
        assert xerr <= 1e-12
