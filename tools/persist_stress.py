#!/usr/bin/env python3
"""Repeated solves across host-bootstrapped processes on one GPU: a rare race
in the multi-rank protocol (the in-kernel peer all-reduce, the in-launch pull
of r's ghost rows, the persistent launch's per-iteration slots) would show as
a solve whose bits differ from the first one's, or as an expired wait (a
resident retry). Every rank solves each size `--solves` times and compares
(niters, normr, trace, x) with its first solve, bit for bit.

    python -m torch.distributed.run --nproc-per-node 2 tools/persist_stress.py OUT [--solves 200]
    python -m torch.distributed.run --nproc-per-node 8 tools/persist_stress.py OUT --dims 16,16,16
    python tools/persist_stress.py OUT --dims 100,100,100 --solves 1000     (one rank)

Writes OUT/stress_rank<r>.json; rank 0 prints a one-line summary."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import load_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--solves", type=int, default=200)
    ap.add_argument("--dims", default="40,36,30;80,80,80", help="';'-separated nx,ny,nz per rank")
    ap.add_argument("--max-iter", type=int, default=500)
    ap.add_argument("--stencil", type=int, default=27)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    hp = load_pkg()
    dev = 0
    torch.cuda.set_device(dev)
    hp.set_device(dev)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        hp.comm_init_host(world, rank)
    else:  # one process (python tools/persist_stress.py OUT): the single-rank launches
        class _One:
            @staticmethod
            def barrier():
                pass
        dist = _One
    res = {"rank": rank, "world": world, "cases": {}}
    for spec in args.dims.split(";"):
        dims = tuple(int(v) for v in spec.split(","))
        M = hp.Matrix.generate(*dims, use_7pt=args.stencil == 7)
        b, _, _ = M.vectors()
        n = M.info()["nrow"]
        x = torch.zeros(n, dtype=torch.float64, device=f"cuda:{dev}")
        first, diff, t0 = None, 0, None
        dist.barrier()
        t0 = time.perf_counter()
        for i in range(args.solves):
            x.zero_()
            _, it, nr, _ = hp.HPCCG(M, b, x, max_iter=args.max_iter, device=True)
            got = (it, nr, M.last_trace().tobytes(), x.cpu().numpy().tobytes())
            if first is None:
                first = got
            elif got != first:
                diff += 1
        dist.barrier()
        dt = time.perf_counter() - t0
        res["cases"]["x".join(map(str, dims))] = {
            "solves": args.solves, "differing": diff, "niters": first[0], "normr": first[1].hex(),
            "retries": M.get_option("resident_retries"), "resident_update": M.get_option("resident_update"),
            "peer_allreduce": M.get_option("peer_allreduce"), "halo_pull": M.get_option("halo_pull"),
            "us_per_iter": dt / args.solves / max(1, first[0]) * 1e6,
            "x_err": float(np.max(np.abs(np.frombuffer(first[3]) - 1.0)))}
        M.close()
    os.makedirs(args.out, exist_ok=True)
    with open(os.path.join(args.out, f"stress_rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    if rank == 0:
        allr = [json.load(open(os.path.join(args.out, f"stress_rank{r}.json"))) for r in range(world)]
        summ = {}
        for name in res["cases"]:
            cs = [d["cases"][name] for d in allr]
            summ[name] = {"world": world, "solves": cs[0]["solves"], "differing_max": max(c["differing"] for c in cs),
                          "retries_max": max(c["retries"] for c in cs),
                          "same_over_ranks": len({(c["niters"], c["normr"]) for c in cs}) == 1,
                          "resident_update": cs[0]["resident_update"], "us_per_iter": round(cs[0]["us_per_iter"], 2),
                          "x_err_max": max(c["x_err"] for c in cs)}
        print(json.dumps(summ), flush=True)
    if world > 1:
        hp.comm_destroy()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
