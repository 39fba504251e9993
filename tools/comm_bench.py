#!/usr/bin/env python3
"""What the RCCL rank path adds per CG iteration, measured on ONE GPU
(diagnostic, not a scaling number): a 1-rank RCCL communicator and
force_comm = 1 (p.Ap and r.r through ncclAllReduce) or 2 (also the
multi-rank iteration: halo fork/join on the second stream, a plane-sized
ncclSend/ncclRecv to itself), against the plain single-GPU solve. One JSON
line per (force_comm, use_graph).

usage: tools/comm_bench.py [--n 200] [--steps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import load_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--max-iter", type=int, default=500)
    ap.add_argument("--7pt", dest="s7", action="store_true")
    ap.add_argument("--variants", default="0:1,1:1,2:1,2:0",
                    help="force_comm:use_graph pairs, optionally :spmv_kernel[:peer_allreduce[:halo_pull]] (-1 auto)")
    args = ap.parse_args()
    import torch
    hp = load_pkg()
    hp.set_device(0)
    hp.comm_init(hp.comm_unique_id(), 1, 0)
    try:
        n3 = args.n ** 3
        M = hp.Matrix.generate(args.n, args.n, args.n, use_7pt=args.s7)
        b = M.vectors()[0]
        x = torch.zeros(n3, dtype=torch.float64, device="cuda:0")
        base = None
        traces = {}
        for v in args.variants.split(","):
            f = [int(t) for t in v.split(":")]
            fc, graph = f[:2]
            M.set_option("spmv_kernel", f[2] if len(f) > 2 else -1)
            M.set_option("peer_allreduce", f[3] if len(f) > 3 else -1)
            M.set_option("halo_pull", f[4] if len(f) > 4 else -1)
            M.set_option("force_comm", fc)
            M.set_option("use_graph", graph)

            def solve():
                x.zero_()
                return hp.HPCCG(M, b, x, max_iter=args.max_iter, device=True)[1]

            solve()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                it = solve()
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / args.steps / it * 1e6
            if base is None:
                base = us
            traces[v] = M.last_trace().tobytes()
            print(json.dumps({"n": args.n, "stencil": 7 if args.s7 else 27, "force_comm": fc,
                              "use_graph": graph, "us_per_iter": round(us, 2),
                              "added_us_per_iter": round(us - base, 2),
                              "graph_used": M.get_option("graph_used"),
                              "kernel": M.get_option("spmv_kernel"), "fuse_p": M.get_option("fuse_p"),
                              "rhalo": M.get_option("rhalo"),
                              "peer_allreduce": M.get_option("peer_allreduce"),
                              "halo_pull": M.get_option("halo_pull"),
                              "fuse_update": M.get_option("fuse_update"),
                              "niters": it,
                              "trace_equal_first": traces[v] == next(iter(traces.values()))}), flush=True)
        M.close()
    finally:
        hp.comm_destroy()


if __name__ == "__main__":
    main()
