"""One rank of the host-bootstrapped 2-process job (tests/test_gpu_hostcomm.py):
two processes share GPU 0, torch.distributed (gloo) carries the setup
exchanges through hpccg_hip_comm_init_host, and the CG iteration runs the
default multi-rank transport for real between the processes -- IPC-mapped
peer mailboxes (the in-kernel all-reduce of ddot.cpp:75-85) and r's ghost
planes pulled from the other process's memory (exchange_externals.cpp:
51-131). Writes <out>/rank<r>.json (+ .npy vectors) for the test to check.

    python -m torch.distributed.run --nproc-per-node 2 tests/hostcomm_worker.py <out_dir>
    python -m torch.distributed.run --nproc-per-node 8 tests/hostcomm_worker.py <out_dir> eight

"eight": the 8-process job (the world size of the driver's 8-GPU run) on one
GPU: the reference's 8-rank golden (27pt_16x16x16_x8ranks) through the default
transport, every rank's mailbox mapped by the seven others.
"""
import json
import os
import sys
import time
import traceback

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from conftest import RTRANS_RTOL_MULTI, check_final, check_trace, kat2_rr0, load_pkg, solve_case, unhex  # noqa: E402


FUZZ_SEED = 2606
FUZZ_CASES = 16


def fuzz_cases(seed=FUZZ_SEED, count=FUZZ_CASES):
    """(i, (nx, ny, nz per rank), 7-pt?, max_iter) for the 2-process fuzz:
    thin and odd slabs, 1- and 2-wide axes, both stencils, short and long
    solves, sizes from one slice up to ones whose two ranks' pair blocks
    no longer fit the GPU together (the per-iteration launches then)."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(count):
        s7 = bool(rng.integers(2))
        nx, ny = (int(v) for v in rng.integers(1, 41, size=2))
        nz = int(rng.integers(1, 25))
        if i % 5 == 1:
            nx = 1
        elif i % 5 == 2:
            ny = 2
        out.append((i, (nx, ny, nz), s7, int(rng.integers(1, 151))))
    # and three larger slabs: 2 x 240 pair blocks (persistent across the
    # processes), 2 x 563 (more than the GPU holds at once: the per-iteration
    # launches), 7-pt 2 x 74^3
    for j, (dims, s7, it) in enumerate((((64, 64, 60), False, 120), ((80, 80, 90), False, 60),
                                        ((74, 74, 74), True, 90))):
        out.append((count + j, dims, s7, it))
    return out


def fuzz_x0(n, rank):
    """A nonzero x0 of this rank's rows, a function of the global row: the
    in-process group builds the same vectors."""
    g = np.arange(n, dtype=np.float64) + rank * n
    return 0.125 * (np.remainder(g * 7.0, 11.0) - 5.0)


def main():
    import torch
    import torch.distributed as dist
    out_dir = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    hp = load_pkg()
    dev = int(os.environ.get("LOCAL_RANK", rank)) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    hp.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    hp.comm_init_host(world, rank)
    res = {"rank": rank, "device": dev, "comm_mode": hp.comm_mode(), "pci": hp.runtime_info()["pci_bus_id"]}
    with open(os.path.join(HERE, "golden", "golden.json")) as f:
        golden = json.load(f)

    def solve(M, b, max_iter=500, tol=0.0):
        n = M.info()["nrow"]
        x = torch.zeros(n, dtype=torch.float64, device=f"cuda:{dev}")
        _, it, nr, times = hp.HPCCG(M, b, x, max_iter=max_iter, tolerance=tol, device=True)
        return it, nr, M.last_trace().copy(), x.cpu().numpy(), times

    def transport(M):
        return {k: M.get_option(k) for k in ("peer_allreduce", "halo_pull", "rhalo", "fuse_update", "spmv_kernel",
                                             "peer_auto_ok", "pull_auto_ok", "proto_auto_ok", "graph_used",
                                             "resident_update", "persist_auto_ok", "resident_retries")}

    def case(name, fn):
        t0 = time.time()
        try:
            r = fn()
            r["ok"] = True
        except Exception as e:
            r = {"ok": False, "error": f"{type(e).__name__}: {e}", "tb": traceback.format_exc()[-3000:]}
        r["seconds"] = round(time.time() - t0, 3)
        res[name] = r
        dist.barrier()

    # 1-2: the reference's 2-rank goldens (the z-stacked global problem solved by
    # the unmodified reference HPCCG(), tests/golden/make_golden.py)
    def golden_case(gname):
        c = solve_case(golden, gname)
        assert c["ranks"] == world
        M = hp.Matrix.generate(c["nx"], c["ny"], c["nz"], use_7pt=c["use_7pt"])
        b, _, _ = M.vectors()
        it, nr, tr, x, times = solve(M, b)
        out = {"transport": transport(M), "niters": it, "normr": nr.hex(), "trace0": tr[0].hex()}
        ref_tr = [unhex(t) for t in c["trace_normr"]]
        rr = c["runs"]["500"]
        assert tr[0] == ref_tr[0]
        out["checked"] = check_trace(tr, ref_tr, RTRANS_RTOL_MULTI)
        assert out["checked"] >= 5
        check_final(it, nr, tr, rr["niters"], unhex(rr["normr"]), ref_tr, 500)
        out["x_err"] = float(np.max(np.abs(x - 1.0)))
        assert out["x_err"] <= 1e-12
        out["halo_s"], out["allreduce_s"] = times[5], times[4]
        # the same solve with k_pull launches, and eagerly: the same bits
        same = (it, nr, tr.tobytes(), x.tobytes())
        M.set_option("halo_pull", 1)
        it1, nr1, tr1, x1, _ = solve(M, b)
        out["kpull_same"] = (it1, nr1, tr1.tobytes(), x1.tobytes()) == same
        M.set_option("halo_pull", -1)
        M.set_option("use_graph", 0)
        it2, nr2, tr2, x2, _ = solve(M, b)
        out["eager_same"] = (it2, nr2, tr2.tobytes(), x2.tobytes()) == same
        M.close()
        return out

    if len(sys.argv) > 2 and sys.argv[2] == "eight":
        case("golden27x8", lambda: golden_case("27pt_16x16x16_x8ranks"))
        return finish(res, out_dir, rank, hp, dist)
    if len(sys.argv) > 2 and sys.argv[2] == "fuzz":
        # seeded random 2-process cases (tests/test_gpu_hostcomm.py::test_hostcomm_fuzz
        # solves each with the in-process group and the oracle)
        for i, dims, s7, max_iter in fuzz_cases():
            def one(dims=dims, s7=s7, max_iter=max_iter, i=i):
                M = hp.Matrix.generate(*dims, use_7pt=s7)
                b, _, _ = M.vectors()
                n = M.info()["nrow"]
                x = torch.from_numpy(fuzz_x0(n, rank)).to(f"cuda:{dev}")
                _, it, nr, _ = hp.HPCCG(M, b, x, max_iter=max_iter, device=True)
                np.savez(os.path.join(out_dir, f"fuzz_c{i}_rank{rank}.npz"), trace=M.last_trace().copy(),
                         x=x.cpu().numpy())
                out = {"transport": transport(M), "niters": it, "normr": nr.hex()}
                M.close()
                return out
            case(f"fuzz{i}", one)
        return finish(res, out_dir, rank, hp, dist)
    case("golden27", lambda: golden_case("27pt_8x8x8_x2ranks"))
    case("golden7", lambda: golden_case("7pt_12x10x8_x2ranks"))

    # 3-4: 2 x 64^3, bits for the in-process group comparison; then one rank
    # withholds a p.Ap partial: both ranks must give up within the spin budget
    # (the other one waits for the missing peer contribution), and the next
    # solve must be bitwise the first
    state = {}

    def bits64():
        M = hp.Matrix.generate(64, 64, 64)
        b, _, _ = M.vectors()
        it, nr, tr, x, _ = solve(M, b)
        np.save(os.path.join(out_dir, f"x64_rank{rank}.npy"), x)
        np.save(os.path.join(out_dir, f"tr64_rank{rank}.npy"), tr)
        state["M"], state["b"], state["first"] = M, b, (it, nr, tr.tobytes(), x.tobytes())
        return {"transport": transport(M), "niters": it, "normr": nr.hex()}

    def bits64x0():
        # a nonzero x0: the prologue's p = x halo is pulled from the other
        # process's x (values, not zeros)
        M, b = state["M"], state["b"]
        n = 64 ** 3
        g = torch.arange(n, dtype=torch.float64, device=f"cuda:{dev}") + rank * n
        x = 0.25 * (torch.remainder(g, 7.0) - 3.0)
        _, it, nr, _ = hp.HPCCG(M, b, x, max_iter=500, device=True)
        np.save(os.path.join(out_dir, f"x64x0_rank{rank}.npy"), x.cpu().numpy())
        np.save(os.path.join(out_dir, f"tr64x0_rank{rank}.npy"), M.last_trace().copy())
        return {"niters": it, "normr": nr.hex()}

    def withhold():
        M, b = state["M"], state["b"]
        budget_us = 200000
        M.set_option("spin_budget_us", budget_us)
        if rank == 0:
            M.set_option("dbg_withhold", 1)
        t0 = time.time()
        err = None
        try:
            solve(M, b)
        except hp.HPCCGError as e:
            err = str(e)
        dt = time.time() - t0
        M.set_option("dbg_withhold", 0)
        M.set_option("spin_budget_us", 1000000)
        it, nr, tr, x, _ = solve(M, b)
        return {"error": err, "seconds_failed": dt, "budget_s": budget_us * 1e-6,
                "after_same": (it, nr, tr.tobytes(), x.tobytes()) == state["first"]}

    case("bits64", bits64)
    case("bits64x0", bits64x0)
    case("withhold", withhold)
    if "M" in state:
        state["M"].close()

    # 5: the kernel-level entry points across the processes: HPC_sparsemv with
    # the host-staged halo (KAT-1: A 1 = b bitwise), ddot all-reduced (KAT-2)
    def kernel_level():
        nx, ny, nz = 12, 10, 8
        M = hp.Matrix.generate(nx, ny, nz)
        n = nx * ny * nz
        ones = torch.ones(n, dtype=torch.float64, device=f"cuda:{dev}")
        y = torch.zeros(n, dtype=torch.float64, device=f"cuda:{dev}")
        hp.HPC_sparsemv(M, ones, y)
        prob = hp.generate_matrix(nx, ny, nz, rank, world)  # the host generator's b of this rank
        kat1 = y.cpu().numpy().tobytes() == prob.b.tobytes()
        prob.close()
        rr = hp.ddot(n, y, y)
        M.close()
        return {"kat1": kat1, "rr": rr, "kat2": float(kat2_rr0(nx, ny, nz * world))}

    case("kernel_level", kernel_level)

    # 6: the collective fallback: rank 1's production-
    # protocol self-test reports a failure (HPCCG_DBG_FAIL_PROTO); every rank
    # must reach the same verdict -- a host-bootstrapped job has no RCCL to
    # fall back to, so the matrix is refused on EVERY rank -- and the next
    # creation, with no failure injected, passes on every rank again
    def fallback():
        out = {}
        if rank == 1:
            os.environ["HPCCG_DBG_FAIL_PROTO"] = "1"
        try:
            M = hp.Matrix.generate(16, 16, 8)
            out["refused"] = None
            M.close()
        except hp.HPCCGError as e:
            out["refused"] = str(e)
        finally:
            os.environ.pop("HPCCG_DBG_FAIL_PROTO", None)
        dist.barrier()
        M = hp.Matrix.generate(16, 16, 8)
        out["after"] = transport(M)
        M.close()
        return out

    case("fallback", fallback)

    # 7: the persistent launch across the processes: one
    # launch per solve on every rank, the dots summed over the ranks inside it
    # and r's ghost rows pulled at the top of every iteration -- bitwise the
    # per-iteration launches of the same transport (resident_update 0), on the
    # size VERDICT r5 names (2 x 40x36x30) and on 2 x 80^3 (500 pair blocks
    # per rank: both ranks' blocks co-resident on this one GPU), with the
    # iteration times of both forms (emulated: the two ranks share the GPU)
    def persist_case(dims, steps):
        M = hp.Matrix.generate(*dims)
        b, _, _ = M.vectors()
        out = {"transport": transport(M)}
        solve(M, b)  # (warm)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            it, nr, tr, x, _ = solve(M, b)
        dist.barrier()
        out["us_per_iter_persistent"] = (time.perf_counter() - t0) / steps / it * 1e6
        got = (it, nr, tr.tobytes(), x.tobytes())
        out["used"] = M.get_option("resident_update")
        M.set_option("resident_update", 0)
        solve(M, b)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            it0, nr0, tr0, x0, _ = solve(M, b)
        dist.barrier()
        out["us_per_iter_launches"] = (time.perf_counter() - t0) / steps / it0 * 1e6
        out["same"] = (it0, nr0, tr0.tobytes(), x0.tobytes()) == got
        out["niters"], out["normr"] = it, nr.hex()
        out["retries"] = M.get_option("resident_retries")
        M.close()
        return out

    case("persist40", lambda: persist_case((40, 36, 30), 3))

    # the persistent launch across processes over two launch windows (1100
    # iterations: kPersistWindow = 512 per launch; the second launch resumes
    # from the ghost rows and mailbox parities the first left), with a
    # tolerance exit inside the second window and from a nonzero x0: bitwise
    # the per-iteration launches
    def persist_windows():
        M = hp.Matrix.generate(40, 36, 30)
        b, _, _ = M.vectors()
        n = M.info()["nrow"]
        g = torch.arange(n, dtype=torch.float64, device=f"cuda:{dev}") + rank * n
        x0 = 0.125 * (torch.remainder(g, 5.0) - 2.0)

        def run(max_iter, tol=0.0):
            x = x0.clone()
            _, it, nr, _ = hp.HPCCG(M, b, x, max_iter=max_iter, tolerance=tol, device=True)
            return it, nr, M.last_trace().tobytes(), x.cpu().numpy().tobytes()

        out = {"used": M.get_option("resident_update")}
        M.set_option("resident_update", 0)
        ref = run(1100)
        tr = np.frombuffer(ref[2])
        tol = float(tr[700])
        ref_tol = run(1100, tol)
        M.set_option("resident_update", -1)
        got, got_tol = run(1100), run(1100, tol)
        out["same"] = got == ref
        out["same_tol"] = got_tol == ref_tol
        out["niters"], out["niters_tol"] = ref[0], ref_tol[0]
        out["retries"] = M.get_option("resident_retries")
        M.close()
        return out

    case("persist_windows", persist_windows)
    case("persist80", lambda: persist_case((80, 80, 80), 5))

    # 8: rank 1's persistent-launch self-test fails (HPCCG_DBG_FAIL_PERSIST):
    # every rank keeps the in-kernel transport but runs the per-iteration
    # launches (the collective verdict), the same bits
    def persist_fallback():
        if rank == 1:
            os.environ["HPCCG_DBG_FAIL_PERSIST"] = "1"
        try:
            M = hp.Matrix.generate(40, 36, 30)
        finally:
            os.environ.pop("HPCCG_DBG_FAIL_PERSIST", None)
        b, _, _ = M.vectors()
        out = {"transport": transport(M)}
        it, nr, tr, x, _ = solve(M, b)
        out["niters"], out["normr"] = it, nr.hex()
        M.close()
        return out

    case("persist_fallback", persist_fallback)

    # 9: degenerate starts across the processes (tests/test_gpu_edge.py's
    # cases): the persistent launch and the per-iteration launches give the
    # same outcome -- no iteration from a zero or NaN residual, the 0/0 path
    # to niters 2 under a negative tolerance or an infinite b entry -- with the
    # non-finite entry on rank 1's first plane (the rows rank 0 pulls); the
    # NaN partials pass the dot slots and mailboxes without a wait expiring
    def degenerate():
        dims = (40, 36, 30)
        M = hp.Matrix.generate(*dims)
        n = M.info()["nrow"]
        d = f"cuda:{dev}"
        ones = torch.ones(n, dtype=torch.float64, device=d)
        y = torch.zeros(n, dtype=torch.float64, device=d)
        hp.HPC_sparsemv(M, ones, y)  # this rank's b (KAT-1: A 1 = b bitwise)
        i = 7 if rank == 1 else 0
        runs = {}

        def put(v, val):
            w = y.clone() if v is None else v.clone()
            if rank == 1:
                w[i] = val
            return w

        todo = {"exact": (y, ones, 30, 0.0), "zero_rhs": (torch.zeros_like(y), torch.zeros_like(y), 30, 0.0),
                "exact_negtol": (y, ones, 30, -1.0), "nan_b": (put(None, float("nan")), torch.zeros_like(y), 30, 0.0),
                "nan_x0": (y, put(torch.zeros_like(y), float("nan")), 30, 0.0),
                "inf_x0": (y, put(torch.zeros_like(y), float("inf")), 30, 0.0),
                "inf_b": (put(None, float("-inf")), torch.zeros_like(y), 30, 0.0)}
        out = {"used": M.get_option("resident_update")}
        for form in (-1, 0):
            M.set_option("resident_update", form)
            for name, (bb, x0, mi, tol) in todo.items():
                x = x0.clone()
                _, it, nr, _ = hp.HPCCG(M, bb, x, max_iter=mi, tolerance=tol, device=True)
                xh = x.cpu().numpy()
                rec = (it, nr.hex(), xh.tobytes())
                if form == -1:
                    runs[name] = rec
                    out[name] = {"niters": it, "normr": nr.hex(), "x_nan": int(np.isnan(xh).sum()),
                                 "x_is_x0": bool(np.array_equal(xh, x0.cpu().numpy(), equal_nan=True))}
                else:
                    out[name]["launches_same"] = rec == runs[name]
        out["retries"] = M.get_option("resident_retries")
        out["n"] = n
        M.close()
        return out

    case("degenerate", degenerate)
    finish(res, out_dir, rank, hp, dist)


def finish(res, out_dir, rank, hp, dist):
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    hp.comm_destroy()
    dist.destroy_process_group()
    print(f"HOSTCOMM-WORKER-DONE rank {rank}", flush=True)


if __name__ == "__main__":
    main()
