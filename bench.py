#!/usr/bin/env python3
"""bench.py -- HPCCG on MI355X: CG iterations/s and effective SpMV GB/s.

One *step* = one full HPCCG() solve (HPCCG.cpp:312-402) with max_iter = 500
(499 CG iterations, tolerance 0: main.cpp:187-188) on the 27-point
nx = ny = nz = 200 problem per GPU (BASELINE.json configs[2]), matrix, b and
x resident in HBM before the timed region (device generator).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 200] [--stencil 27]

N > 1: launched by torch.distributed.run, one process per GPU; z-stacked
slabs (local nz fixed, weak scaling), halo + dot all-reduces over RCCL inside
libhpccg_hip.so; torch.distributed (gloo) carries only the control plane
(unique id, barrier, max-over-ranks time).

value = (CG iterations x ranks x K) / max-over-ranks wall time of the K steps
      = 200^3-slab CG iterations per second summed over GPUs (at N = 1:
        plain CG iterations/s).
roofline: the SpMV kernel (84 % of the reference's time);
  achieved = algorithmic bytes of the reference operations it performs
  (12 nnz + 20 n SpMV, 16 n ddot(p, Ap), + 24 n waxpby when the p update is
  fused) per launch / average launch duration from hipEvents on the solver
  stream in the first --event-steps timed steps (launched eagerly; the other
  timed steps replay hipGraphs); peak 8 TB/s.
cpu_baseline: the reference compiled from its own sources (oracle/_ref, OpenMP)
  -- or the oracle port if that build is absent -- on a bounded sample of the
  same problem, rank 0, N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ.setdefault("OMP_NUM_THREADS", "16")
os.environ.setdefault("OMP_PROC_BIND", "close")

ROOT = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def load_pkg():
    import importlib.util
    name = "hpccg_sycl_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "hpccg-sycl_amd",
                                                                    "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(nx, ny, nz, use_7pt, budget_s=15.0):
    """Time the reference (or the oracle port) on the host cores, bounded."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle  # test infrastructure: baseline leg only
    threads = int(os.environ.get("OMP_NUM_THREADS", "16"))
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libhpccg_ref_omp.so")
    # sample: the same matrix, first `iters` CG iterations
    A = oracle.generate(nx, ny, nz, use_7pt=use_7pt)
    probe = 3
    if os.path.exists(ref_so) and not use_7pt:
        kind = "reference"
        M = oracle.ref_from_csr(A, omp=True)
        run = lambda mi: oracle.ref_hpccg(M, A.b, max_iter=mi)  # noqa: E731
    else:
        kind = "port"
        run = lambda mi: oracle.hpccg(A, max_iter=mi, nthreads=threads, trace=False)  # noqa: E731
    # the reference prints residual lines on fd 1: keep bench stdout to one JSON line
    saved = os.dup(1)
    null = os.open(os.devnull, os.O_WRONLY)
    os.dup2(null, 1)
    try:
        t = run(probe + 1)["times"][0]
        per_it = max(t / probe, 1e-6)
        iters = int(max(5, min(500, budget_s / per_it)))
        res = run(iters + 1)
    finally:
        import ctypes
        ctypes.CDLL(None).fflush(None)
        os.dup2(saved, 1)
        os.close(null)
        os.close(saved)
    its = res["niters"] / res["times"][0]
    return {"value": its, "unit": "CG iterations/s", "cores": threads, "kind": kind,
            "sample": f"{nx}x{ny}x{nz} {'7' if use_7pt else '27'}-pt, first {res['niters']} CG "
                      f"iterations of one HPCCG() solve ({res['times'][0]:.1f} s), "
                      f"OpenMP {threads} threads on the GPU box host"}


def matrix_format(v):
    """Matrix image a SpMV variant streams (hpccg_solver.cpp slot_bytes) and
    its bytes per stored slot."""
    if 8960 <= v < 9000:
        return ("SELL-512-A (8 B value per offset-aligned slot, holes 0.0), x from LDS windows shared "
                "by slice pairs"), 8.0
    if 8900 <= v < 8960:
        return "SELL-512-A (8 B value per offset-aligned slot, holes 0.0), x from LDS windows", 8.0
    if 8700 <= v < 8900:
        return "SELL-512-A (8 B value per offset-aligned slot, holes 0.0; x read at per-slice offsets)", 8.0
    if v >= 8000:
        return "SELL-512-P (8 B value per slot + 1-byte row-pattern id per row)", 8.0
    if v >= 7000:
        return "SELL-512-V4 (1-byte (offset, value) codes, 4-slot chunks)", 1.0
    if v >= 5000:
        return "SELL-512-V (1-byte (offset, value) codes)", 1.0
    if v >= 4000:
        return "SELL-512-C + LDS x windows (8 B value + 1-byte offset code)", 9.0
    if v >= 3000:
        return "SELL-512-C (8 B value + 1-byte offset code)", 9.0
    if v >= 2000:
        return "SELL-512-L (8 B value + 16-bit window index)", 10.0
    return "SELL-512 (8 B value + int32 column)", 12.0


def spmv_kernel_family(v):
    """Kernel template a SpMV variant launches (hpccg_kernels.hip launch_cg_spmv)."""
    if 8960 <= v < 9000:
        return "k_spmv_la2"
    if 8900 <= v < 8960:
        return "k_spmv_la"
    if 8700 <= v < 8900:
        return "k_spmv_pa"
    if 8500 <= v < 8700:
        return "k_spmv_pp"
    if 8000 <= v < 8500:
        return "k_spmv_lp"
    return None


def pmc_traffic(tag, fused_p, variant):
    """HBM bytes per SpMV launch from the committed rocprofv3 PMC summary of
    the same kernel configuration (profiles/pmc_<tag>.json), else None."""
    import re
    path = os.path.join(ROOT, "profiles", f"pmc_{tag}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    if bool(d.get("fuse_p", False)) != bool(fused_p):
        return None
    fam = spmv_kernel_family(variant)
    m = re.search(r"(k_spmv\w*)<", d.get("kernel", ""))
    if fam is not None and (m is None or m.group(1) != fam):
        return None  # the summary measured another kernel
    return d.get("spmv_hbm_bytes_per_launch")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=200, help="nx = ny = nz per GPU")
    ap.add_argument("--stencil", type=int, default=27, choices=[27, 7])
    ap.add_argument("--max-iter", type=int, default=500)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--variant", type=int, default=-1, help="SpMV kernel variant (-1 auto)")
    ap.add_argument("--fuse-p", type=int, default=-1, help="p update inside the SpMV (-1 default)")
    ap.add_argument("--fold", type=int, default=-1, help="last-block dot completion (-1 default)")
    ap.add_argument("--graph-chunk", type=int, default=-1, help="CG iterations per hipGraph (-1 default)")
    ap.add_argument("--redund", type=int, default=-1,
                    help="consumers complete the dot products themselves (-1 default)")
    ap.add_argument("--x-defer", type=int, default=-1, help="batched x update (-1 default)")
    ap.add_argument("--update-early", type=int, default=-1,
                    help="loop update loads Ap and r before the iteration test (-1 default)")
    ap.add_argument("--pap-in-update", type=int, default=-1,
                    help="the loop update sums the SpMV's p.Ap partials itself (-1 default)")
    ap.add_argument("--update-slices", type=int, default=-1,
                    help="slices per loop-update workgroup: 1, 2, 4, 8 (-1 default)")
    ap.add_argument("--x-ring", type=int, default=-1,
                    help="x-update deferral depth = p ring length (-1 default)")
    ap.add_argument("--resident-mb", type=int, default=-1,
                    help="MB of the matrix image streamed with default-policy loads (-1 default)")
    ap.add_argument("--rev-update", type=int, default=-1,
                    help="update kernel walks slices backwards (-1 default)")
    ap.add_argument("--value-codes", type=int, default=0,
                    help="1: headline with SELL-512-V (values from a per-slice dictionary); default 0 "
                         "streams every stored value and reports SELL-512-V as a secondary figure")
    ap.add_argument("--no-secondary", action="store_true", help="skip the SELL-512-V secondary run")
    ap.add_argument("--event-steps", type=int, default=1,
                    help="timed steps launched eagerly with hipEvents around every SpMV (the "
                         "roofline's kernel time); the other timed steps replay hipGraphs")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    hp = load_pkg()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    torch.cuda.set_device(local_rank)
    hp.set_device(local_rank)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        obj = [hp.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        hp.comm_init(obj[0], world, rank)

    n = args.n
    use_7pt = args.stencil == 7
    t0 = time.time()
    M = hp.Matrix.generate(n, n, n, use_7pt=use_7pt)
    info = M.info()
    if args.variant >= 0:
        M.set_option("spmv_variant", args.variant)
    if args.fuse_p >= 0:
        M.set_option("fuse_p", args.fuse_p)
    if args.fold >= 0:
        M.set_option("fold", args.fold)
    if args.redund >= 0:
        M.set_option("redund", args.redund)
    if args.graph_chunk > 0:
        M.set_option("graph_chunk", args.graph_chunk)
    if args.x_defer >= 0:
        M.set_option("x_defer", args.x_defer)
    if args.update_slices > 0:
        M.set_option("update_slices", args.update_slices)
    if args.update_early >= 0:
        M.set_option("update_early", args.update_early)
    if args.pap_in_update >= 0:
        M.set_option("pap_in_update", args.pap_in_update)
    if args.x_ring > 0:
        M.set_option("x_ring", args.x_ring)
    if args.rev_update >= 0:
        M.set_option("rev_update", args.rev_update)
    if args.resident_mb >= 0:
        M.set_option("resident_mb", args.resident_mb)
    if args.value_codes:
        M.set_option("value_codes", 1)
    b, x0, _ = M.vectors()
    nrow = n * n * n
    x = torch.zeros(nrow, dtype=torch.float64, device=f"cuda:{local_rank}")
    torch.cuda.synchronize()
    log(f"[rank {rank}] setup {time.time() - t0:.2f}s nnz={info['nnz']} slots={info['slots']} "
        f"variant={info['spmv_variant']}")

    def step(events):
        M.set_option("event_timing", 1 if events else 0)
        x.zero_()
        return hp.HPCCG(M, b, x, max_iter=args.max_iter, device=True)

    cold_s = None
    for i in range(args.warmup):
        t0 = time.perf_counter()
        step(i == 0)
        if i == 0:
            cold_s = time.perf_counter() - t0  # first solve: graph build, cold caches

    def barrier():
        if world > 1:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    niters_total = 0
    spmv_ms = spmv_n = upd_ms = upd_n = 0.0
    times_acc = [0.0] * 7
    step_s = []
    for i in range(args.steps):
        ev = i < args.event_steps
        t0 = time.perf_counter()
        _, it, nr, times = step(ev)
        step_s.append(time.perf_counter() - t0)
        niters_total += it
        if ev:
            kt = M.kernel_times()
            spmv_ms += kt["spmv_ms"]
            spmv_n += kt["spmv_launches"]
            upd_ms += kt["update_ms"]
            upd_n += kt["update_launches"]
        for i in range(7):
            times_acc[i] += times[i]
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    # outside the timed region: the last solve's answer (xexact = 1, generate_matrix.cpp:286)
    # and residual reduction, max over ranks -- a wrong multi-rank exchange shows here
    tr = M.last_trace()
    chk = torch.tensor([(x - 1.0).abs().max().item(), float(nr / tr[0]) if tr[0] > 0 else 0.0],
                       dtype=torch.float64)
    if world > 1:
        dist.all_reduce(chk, op=dist.ReduceOp.MAX)

    # Algorithmic bytes of the reference operations the SpMV kernel performs
    # (fused kernels are credited with the unfused bytes):
    # HPC_sparsemv 12 nnz + 20 n, ddot(p, Ap) 16 n, and with fuse_p the
    # waxpby p = r + beta p, 24 n.
    fused_p = M.get_option("fuse_p")
    spmv_bytes = 12.0 * info["nnz"] + 20.0 * nrow + 16.0 * nrow + (24.0 * nrow if fused_p else 0.0)
    if spmv_n > 0:
        spmv_avg_s = spmv_ms / spmv_n * 1e-3
        timing_src = ("hipEvent pairs around every SpMV launch on the solver stream, %d of the "
                      "%d timed steps (the others replay hipGraphs)" % (args.event_steps, args.steps))
    else:  # graph mode: device-clock stamps (SPARSEMV class time / calls)
        spmv_avg_s = times_acc[3] / max(1, niters_total + args.steps)
        timing_src = "s_memrealtime stamps (graph mode)"
    achieved = spmv_bytes / spmv_avg_s / 1e9
    it_per_s = niters_total / elapsed  # per rank: every rank runs the same iterations
    value = it_per_s * world
    ms_per_step = elapsed / args.steps * 1e3
    iter_bytes = 12.0 * info["nnz"] + 116.0 * nrow  # unfused reference sequence, SURVEY 8(d)

    # Secondary figure (not `value`): the same solves with SELL-512-V, whose
    # per-slice (offset, value) dictionary replaces the streamed values.
    secondary = None
    if not args.value_codes and not args.no_secondary and M.get_option("value_codes_available"):
        keep_variant = M.get_option("spmv_variant")
        M.set_option("value_codes", 1)
        step(False)  # warm-up: graph build for the new kernel
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        it2 = 0
        for i in range(args.steps):
            it2 += step(i < args.event_steps)[1]
            if i < args.event_steps:
                kt2 = M.kernel_times()
        torch.cuda.synchronize()
        barrier()
        el2 = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el2], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el2 = t.item()
        xerr2 = (x - 1.0).abs().max().item()
        secondary = {
            "format": "SELL-512-V (1-byte codes of per-slice (column - row, value) pairs; lossless, "
                      "bitwise-equal results; not the headline: it does not stream the stored values)",
            "value": round(it2 / el2 * world, 3),
            "spmv_variant": M.get_option("spmv_variant"),
            "spmv_avg_us": round(kt2["spmv_ms"] / max(1, kt2["spmv_launches"]) * 1e3, 2)
            if args.event_steps > 0 else None,
            "x_minus_xexact_inf": xerr2,
        }
        M.set_option("value_codes", 0)
        M.set_option("spmv_variant", keep_variant)

    if rank == 0:
        out = {
            "metric": "CG iterations/sec + effective SpMV GB/s (% HBM peak), 27-pt nx=ny=nz=200",
            "value": round(value, 3),
            "unit": "CG iterations/s (per-GPU %d^3 slab iterations, summed over GPUs)" % n,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (generate_matrix stencil on the device; deterministic, no RNG)",
            "config": {
                "workload": f"HPCCG solve, {args.stencil}-pt {n}x{n}x{n} per GPU, z-stacked, "
                            f"max_iter={args.max_iter} (499 CG iterations), tolerance 0",
                "nx": n, "ny": n, "nz_per_gpu": n, "stencil": args.stencil,
                "max_iter": args.max_iter, "parallelism": f"z-slab x{world} (RCCL)",
                "nnz_per_gpu": info["nnz"], "sell_slots_per_gpu": info["slots"],
                "spmv_variant": M.get_option("spmv_variant"),
                "matrix_format": matrix_format(M.get_option("spmv_variant"))[0],
                "matrix_bytes_per_slot": matrix_format(M.get_option("spmv_variant"))[1],
                "options": {k: M.get_option(k) for k in ("fuse_p", "fold", "update_slices", "update_early", "pap_in_update", "x_defer", "x_ring", "rev_update",
                                                         "resident_mb", "overlap", "value_codes")},
            },
            "cg_iterations_per_s_global": round(it_per_s, 3),
            "spmv_effective_gbs": round(achieved, 1),
            "spmv_frac_hbm_peak": round(achieved / HBM_PEAK_GBS, 4),
            "iteration_effective_gbs": round(iter_bytes * it_per_s / 1e9, 1),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": pmc_traffic(f"spmv_{args.stencil}pt_{n}", fused_p,
                                       M.get_option("spmv_variant")),
                "kernel": "SpMV variant %d, %s + p.Ap%s" % (M.get_option("spmv_variant"),
                                                           matrix_format(M.get_option("spmv_variant"))[0],
                                                           " + p = r + beta p" if fused_p else ""),
                "bytes_formula": "12 nnz + 20 n (SpMV) + 16 n (ddot p.Ap)" + (" + 24 n (waxpby p)" if fused_p else ""),
                "bytes_per_launch": spmv_bytes,
                "avg_launch_us": round(spmv_avg_s * 1e6, 2),
                "timing": timing_src,
            },
            "value_coded_secondary": secondary,
            "update_kernel_avg_us": round(upd_ms / upd_n * 1e3, 2) if upd_n else None,
            "check": {"x_minus_xexact_inf": chk[0].item(), "final_normr_over_initial": chk[1].item(),
                      "niters_per_solve": it},
            # per-solve wall times on rank 0 (first/cold and median of the solves);
            # event steps launch eagerly with hipEvents and are slower than the graph replays
            "solve_ms": {"cold": round(cold_s * 1e3, 3) if cold_s is not None else None,
                         "median": round(sorted(step_s)[len(step_s) // 2] * 1e3, 3),
                         "min": round(min(step_s) * 1e3, 3), "max": round(max(step_s) * 1e3, 3),
                         "median_graph_replay": round(sorted(step_s[args.event_steps:])[
                             len(step_s[args.event_steps:]) // 2] * 1e3, 3)
                         if len(step_s) > args.event_steps else None},
            "times_per_step_s": {"total": times_acc[0] / args.steps,
                                 "ddot": times_acc[1] / args.steps,
                                 "waxpby": times_acc[2] / args.steps,
                                 "sparsemv": times_acc[3] / args.steps,
                                 "allreduce": times_acc[4] / args.steps,
                                 "halo": times_acc[5] / args.steps},
            "cpu_baseline": None,
        }
        rf = out["roofline"]
        if rf["traffic"]:
            # the bytes the chip moved (PMC) over the same launch time: the
            # credited formula counts 12 B per nonzero and unfused vector passes,
            # more than SELL-512-P + fusion stream, so frac can pass 1.0
            rf["traffic_gbs"] = round(rf["traffic"] / spmv_avg_s / 1e9, 1)
            rf["traffic_frac"] = round(rf["traffic_gbs"] / HBM_PEAK_GBS, 4)
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(n, n, n, use_7pt)
            except Exception as e:  # reported, never silently replaced
                out["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)

    M.close()
    if world > 1:
        hp.comm_destroy()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
