"""N > 1 path on CPU (gloo, world_size 2 and 3).

Each rank uses the library's own host-side pieces exactly as the GPU path
does -- per-rank generator (generate_matrix.cpp:225-229 z-slabs), halo plan
from the column range, the slab plan from the all-gathered {nrow, ghost_lo,
ghost_hi, start_row} (hpccg_slab_plan), the SELL-512 image with
ghost-localised columns (hpccg_sell_build) -- and then emulates the device CG
with the same halo offsets the library gives RCCL (enqueue_halo in
hpccg_solver.cpp) and the same all-reduced recurrence (cg_run / hist logic in
hpccg_kernels.hip). The oracle is the global serial reference run of the
z-stacked problem ("Multi-GPU oracle"), tolerance 1e-7 on rtrans.
"""
import math
import os
import socket

import numpy as np
import pytest

from conftest import (RTRANS_RTOL_MULTI, check_final, check_trace, load_pkg, solve_case, unhex)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spmv_sell(sb, sc, sv, pext, n):
    y = np.zeros(((n + 511) // 512) * 512)
    for s in range(len(sb) - 1):
        acc = np.zeros(512)
        for j in range(int(sb[s + 1] - sb[s])):
            e0 = (int(sb[s]) + j) * 512
            c = sc[e0:e0 + 512]
            xv = np.where(c >= 0, pext[np.maximum(c, 0)], 0.0)
            acc = acc + sv[e0:e0 + 512] * xv
        y[s * 512:(s + 1) * 512] = acc
    return y[:n]


def _worker(rank, world, port, nx, ny, nz, use_7pt, max_iter, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hp = load_pkg()
        n = nx * ny * nz
        prob = hp.generate_matrix(nx, ny, nz, rank=rank, size=world, use_7pt=use_7pt)
        rp, cols, vals = prob.to_csr()
        start, total = rank * n, n * world
        plan = hp.halo_plan(rp, cols, start, total)
        glo, ghi = plan["ghost_lo"], plan["ghost_hi"]
        info = torch.tensor([n, glo, ghi, start], dtype=torch.int32)
        gathered = [torch.zeros(4, dtype=torch.int32) for _ in range(world)]
        dist.all_gather(gathered, info)
        allinfo = torch.cat(gathered).numpy()
        send_lo, send_hi = hp.slab_plan(world, rank, allinfo)
        sb, sc, sv = hp.sell_build(rp, cols, vals, col_base=start - glo, ncol_ext=glo + n + ghi)

        pext = np.zeros(glo + n + ghi)
        P = slice(glo, glo + n)  # local rows of p inside [ghost_lo | n | ghost_hi]

        def halo():
            # enqueue_halo: recv(p - ghost_lo, ghost_lo, r-1); send(p, send_lo, r-1);
            #               recv(p + n, ghost_hi, r+1); send(p + n - send_hi, send_hi, r+1)
            reqs, bufs = [], []
            if rank > 0:
                lo = torch.zeros(glo, dtype=torch.float64)
                reqs.append(dist.irecv(lo, rank - 1))
                bufs.append(("lo", lo))
                reqs.append(dist.isend(torch.from_numpy(pext[glo:glo + send_lo].copy()), rank - 1))
            if rank < world - 1:
                hi = torch.zeros(ghi, dtype=torch.float64)
                reqs.append(dist.irecv(hi, rank + 1))
                bufs.append(("hi", hi))
                reqs.append(dist.isend(torch.from_numpy(pext[glo + n - send_hi:glo + n].copy()),
                                       rank + 1))
            for r in reqs:
                r.wait()
            for which, t in bufs:
                if which == "lo":
                    pext[0:glo] = t.numpy()
                else:
                    pext[glo + n:glo + n + ghi] = t.numpy()

        def allsum(v):
            t = torch.tensor([v], dtype=torch.float64)
            dist.all_reduce(t)
            return t.item()

        b = prob.b
        x = np.zeros(n)
        pext[P] = x + 0.0 * x
        halo()
        Ap = _spmv_sell(sb, sc, sv, pext, n)
        r = b + (-1.0) * Ap
        rr = allsum(float(np.dot(r, r)))
        hist = {}
        trace = [math.sqrt(rr)]
        niters = 0
        for k in range(1, max_iter):
            chk = rr if k == 1 else hist[k - 2]  # cg_run: normr of iteration k-1
            if not math.sqrt(chk) > 0.0:
                break
            if k == 1:
                pext[P] = r + 0.0 * r
            else:
                pext[P] = r + (rr / hist[k - 2]) * pext[P]
            hist[k - 1] = rr
            halo()
            Ap = _spmv_sell(sb, sc, sv, pext, n)
            alpha = rr / allsum(float(np.dot(pext[P], Ap)))
            x = x + alpha * pext[P]
            r = r + (-alpha) * Ap
            rr = allsum(float(np.dot(r, r)))
            niters = k
            trace.append(math.sqrt(hist[k - 1]))
        err = allsum(0.0)  # keep collectives aligned
        q.put((rank, niters, trace, float(np.max(np.abs(x - 1.0))), (send_lo, send_hi, glo, ghi),
               err))
    finally:
        dist.destroy_process_group()


def _run(world, nx, ny, nz, use_7pt, max_iter):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, nx, ny, nz, use_7pt, max_iter, q))
          for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out)


@pytest.mark.parametrize("name,max_iter", [("27pt_8x8x8_x2ranks", 500),
                                           ("7pt_12x10x8_x2ranks", 500)])
def test_two_rank_slab_cg_matches_global_reference(golden, name, max_iter):
    c = solve_case(golden, name)
    out = _run(c["ranks"], c["nx"], c["ny"], c["nz"], c["use_7pt"], max_iter)
    nxy = c["nx"] * c["ny"]
    # plan: rank 0 sends its top plane up, rank 1 its bottom plane down
    assert out[0][4] == (0, nxy, 0, nxy)
    assert out[1][4] == (nxy, 0, nxy, 0)
    ref_tr = [unhex(t) for t in c["trace_normr"]]
    rr = c["runs"]["500"]
    for rank, niters, trace, xerr, _, _ in out:
        assert trace == out[0][2]  # every rank holds the same all-reduced scalars
        assert trace[0] == ref_tr[0]
        assert check_trace(trace, ref_tr, RTRANS_RTOL_MULTI) >= 5
        check_final(niters, trace[-1], np.array(trace), rr["niters"], unhex(rr["normr"]), ref_tr,
                    max_iter)
        assert xerr <= 1e-12


def test_three_rank_plan_interior_rank():
    out = _run(3, 6, 5, 4, False, 40)
    nxy = 30
    assert out[1][4] == (nxy, nxy, nxy, nxy)  # interior: both neighbours
    assert out[0][2] == out[1][2] == out[2][2]
    import oracle
    ref = oracle.hpccg(oracle.generate(6, 5, 12), max_iter=40)
    assert check_trace(out[0][2], ref["trace"], RTRANS_RTOL_MULTI) >= 5


@pytest.mark.parametrize("world", [2, 3, 5])
@pytest.mark.parametrize("use_7pt", [False, True])
def test_pull_halo_contract(world, use_7pt):
    """The halo pull (k_pull) reads rank r-1's last ghost_lo(r)
    rows and rank r+1's first ghost_hi(r) rows of r; the update writes exactly
    the rows the slab plan sends (send_hi(r-1), send_lo(r+1)) write-through.
    For the z-slab plan those must coincide: every pulled row is a sent row,
    and the pull moves what RCCL's send/recv would."""
    hp = load_pkg()
    nx, ny, nz = 7, 5, 4
    n = nx * ny * nz
    info = []
    for r in range(world):
        prob = hp.generate_matrix(nx, ny, nz, rank=r, size=world, use_7pt=use_7pt)
        rp, cols, _ = prob.to_csr()
        plan = hp.halo_plan(rp, cols, r * n, n * world)
        info += [n, plan["ghost_lo"], plan["ghost_hi"], r * n]
        prob.close()
    info = np.array(info, dtype=np.int32)
    sends = [hp.slab_plan(world, r, info) for r in range(world)]
    for r in range(world):
        glo, ghi = info[4 * r + 1], info[4 * r + 2]
        if r > 0:
            assert glo > 0 and glo == sends[r - 1][1]
        else:
            assert glo == 0
        if r < world - 1:
            assert ghi > 0 and ghi == sends[r + 1][0]
        else:
            assert ghi == 0
