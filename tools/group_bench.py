#!/usr/bin/env python3
"""Cost of the multi-rank kernel sequence on ONE GPU (diagnostic, not a
scaling number): P z-slab ranks of n^3 each run as an in-process group on
cuda:0 (k_p_boundary, halo peer copies, rank-ordered scalar sums, eager
launches), against P single-rank solves of the same size. The difference per
iteration is what the multi-rank path adds besides RCCL's own latency.

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
    args = ap.parse_args()
    import torch
    hp = load_pkg()
    hp.set_device(0)
    n3 = args.n ** 3
    Ms = hp.group_generate(args.n, args.n, args.n, args.P)
    bs = [M.vectors()[0] for M in Ms]
    xs = [torch.zeros(n3, dtype=torch.float64, device="cuda:0") for _ in Ms]
    M1 = hp.Matrix.generate(args.n, args.n, args.n)
    b1 = M1.vectors()[0]
    x1 = torch.zeros(n3, dtype=torch.float64, device="cuda:0")

    def group_step():
        for x in xs:
            x.zero_()
        return hp.group_HPCCG(Ms, bs, xs, max_iter=args.max_iter)[1]

    def single_step():
        x1.zero_()
        return hp.HPCCG(M1, b1, x1, max_iter=args.max_iter, device=True)[1]

    out = {}
    for name, fn, reps in (("group", group_step, 1), ("single", single_step, args.P)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        it = 0
        for _ in range(args.steps):
            for _ in range(reps):
                it = fn()
        torch.cuda.synchronize()
        out[name] = (time.perf_counter() - t0) / args.steps / it * 1e6  # us per iteration (all ranks)
    print(json.dumps({"n": args.n, "P": args.P, "group_us_per_iter": round(out["group"], 2),
                      "P_x_single_us_per_iter": round(out["single"], 2),
                      "multi_rank_overhead_us_per_iter": round(out["group"] - out["single"], 2),
                      "variant": Ms[0].get_option("spmv_variant"),
                      "fuse_p": Ms[0].get_option("fuse_p")}))


if __name__ == "__main__":
    main()
