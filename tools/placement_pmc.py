"""one PMC comparison of a slow and a fast 200^3
placement from one process. Phase A solves on the creation placement
(hipMalloc); phase B moves the values image and the p ring to physically
contiguous memory (diag_realloc mode 1 -- diagnostics only: such allocations
corrupted other buffers) and solves again. Each phase runs
`--solves` eager event-timed solves of `--iters` iterations and prints its
median SpMV launch time; run it under rocprofv3 --pmc and split the SpMV
dispatches in order (the first half is phase A).

    rocprofv3 --pmc <counters> -d gpurun_out/pmcX -o run --output-format csv -- \
        python tools/placement_pmc.py --n 200
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import load_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--solves", type=int, default=3)
    ap.add_argument("--mode", type=int, default=1, help="diag_realloc mode of phase B (1 contiguous)")
    args = ap.parse_args()
    import torch
    hp = load_pkg()
    hp.set_device(0)
    M = hp.Matrix.generate(args.n, args.n, args.n)
    b, _, _ = M.vectors()
    x = torch.zeros(args.n ** 3, dtype=torch.float64, device="cuda:0")
    M.set_option("event_timing", 1)

    def phase(tag):
        us = []
        for _ in range(args.solves):
            x.zero_()
            hp.HPCCG(M, b, x, max_iter=args.iters, device=True)
            kt = M.kernel_times()
            us.append(kt["spmv_ms"] / kt["spmv_launches"] * 1e3)
        print(f"PHASE {tag}: SpMV launches {args.solves * args.iters}, median {statistics.median(us):.1f} us "
              f"({', '.join(f'{u:.1f}' for u in us)})", flush=True)

    phase("A creation placement")
    for which in (0, 1):  # values, p ring
        M.diag_realloc(which, args.mode)
    phase(f"B values + ring moved (mode {args.mode})")
    M.close()


if __name__ == "__main__":
    main()
