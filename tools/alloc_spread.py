#!/usr/bin/env python3
"""Spread of the CG rate over fresh allocations in one process: the matrix is
created, solved `--solves` times and released, `--rounds` times; prints the
rate of each round and the SpMV launch average (event-timed solve). Tells a
placement effect (rate changes with the allocation) from box drift.

usage: tools/alloc_spread.py --n 256 --stencil 7 --rounds 6
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
    ap.add_argument("--stencil", type=int, default=27)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--solves", type=int, default=3)
    ap.add_argument("--max-iter", type=int, default=500)
    ap.add_argument("--hold", type=int, default=0, help="keep every round's matrix alive (fresh memory each round)")
    args = ap.parse_args()
    import torch
    hp = load_pkg()
    hp.set_device(0)
    held = []
    for rnd in range(args.rounds):
        M = hp.Matrix.generate(args.n, args.n, args.n, use_7pt=args.stencil == 7)
        b = M.vectors()[0]
        x = torch.zeros(args.n ** 3, dtype=torch.float64, device="cuda:0")

        def solve():
            x.zero_()
            return hp.HPCCG(M, b, x, max_iter=args.max_iter, device=True)[1]

        solve()
        M.set_option("event_timing", 1)
        solve()
        kt = M.kernel_times()
        M.set_option("event_timing", 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.solves):
            it = solve()
        torch.cuda.synchronize()
        rate = it * args.solves / (time.perf_counter() - t0)
        print(json.dumps({"round": rnd, "it_per_s": round(rate, 1),
                          "spmv_us": round(kt["spmv_ms"] / kt["spmv_launches"] * 1e3, 2),
                          "update_us": round(kt["update_ms"] / kt["update_launches"] * 1e3, 2)}), flush=True)
        if args.hold:
            held.append((M, b, x))
        else:
            del b, x
            M.close()
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
