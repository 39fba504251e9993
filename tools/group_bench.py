#!/usr/bin/env python3
"""Cost of the multi-rank iteration on ONE GPU (diagnostic, not a scaling
number): P z-slab ranks of n^3 each run as an in-process group on cuda:0
(k_p_boundary, halo peer copies, rank-ordered scalar sums, graph replay when
use_graph is on), against P single-rank solves of the same size. The
difference per iteration is what the multi-rank path adds besides RCCL's own
latency. One JSON line per group variant (graph on/off x fold).

usage: tools/group_bench.py [--n 200] [--P 2] [--steps 3]
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
    ap.add_argument("--P", type=int, default=2)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--max-iter", type=int, default=500)
    ap.add_argument("--7pt", dest="s7", action="store_true")
    ap.add_argument("--variants", default="1:-1,1:0,0:-1", help="use_graph:fold (fold 0: k_finalize + k_group_sum)")
    ap.add_argument("--no-single", action="store_true")
    args = ap.parse_args()
    import torch
    hp = load_pkg()
    hp.set_device(0)
    n3 = args.n ** 3
    M1 = hp.Matrix.generate(args.n, args.n, args.n, use_7pt=args.s7)
    b1 = M1.vectors()[0]
    x1 = torch.zeros(n3, dtype=torch.float64, device="cuda:0")

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        it = 0
        for _ in range(args.steps):
            for _ in range(reps):
                it = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.steps / it * 1e6  # us per iteration (all ranks)

    def single_step():
        x1.zero_()
        return hp.HPCCG(M1, b1, x1, max_iter=args.max_iter, device=True)[1]

    single = float("nan") if args.no_single else timed(single_step, args.P)
    single_info = {"kernel": M1.get_option("spmv_kernel"), "graph_used": M1.get_option("graph_used"),
                   "fuse_p": M1.get_option("fuse_p")}
    M1.close()
    torch.cuda.empty_cache()

    Ms = hp.group_generate(args.n, args.n, args.n, args.P, use_7pt=args.s7)
    bs = [M.vectors()[0] for M in Ms]
    xs = [torch.zeros(n3, dtype=torch.float64, device="cuda:0") for _ in Ms]

    def group_step():
        for x in xs:
            x.zero_()
        return hp.group_HPCCG(Ms, bs, xs, max_iter=args.max_iter)[1]

    for v in args.variants.split(","):
            f = [int(t) for t in v.split(":")]
            graph, fold = f[0], f[1]
            for M in Ms:
                M.set_option("use_graph", graph)
                M.set_option("fold", fold)
            group = timed(group_step, 1)
            print(json.dumps({
                "n": args.n, "P": args.P, "stencil": 7 if args.s7 else 27,
                "use_graph": graph, "fold": fold, "group_fold": Ms[0].get_option("group_fold"),
                "group_us_per_iter": round(group, 2),
                "P_x_single_us_per_iter": round(single, 2),
                "multi_rank_overhead_us_per_iter": round(group - single, 2),
                "overhead_frac": round(group / single - 1, 4),
                "group": {"kernel": Ms[0].get_option("spmv_kernel"),
                          "graph_used": Ms[0].get_option("graph_used"),
                          "fuse_p": Ms[0].get_option("fuse_p")},
                "single": single_info}), flush=True)


if __name__ == "__main__":
    main()
