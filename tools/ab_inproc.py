#!/usr/bin/env python3
"""Same-process A/B of solver options on one matrix (same allocations, so the
per-process placement spread does not enter): variants run round-robin,
`--reps` rounds of `--solves` solves each; prints the median CG it/s and the
SpMV / update launch averages (one eager event-timed solve per variant).

usage: tools/ab_inproc.py --n 256 --stencil 7 --variants "x_ring=8;x_ring=32"
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import load_pkg  # noqa: E402


def parse(v):
    out = {}
    for kv in filter(None, v.split(",")):
        k, val = kv.split("=")
        out[k.strip()] = int(val)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--stencil", type=int, default=27)
    ap.add_argument("--variants", required=True, help="';'-separated 'key=val,key=val' option sets")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--solves", type=int, default=2)
    ap.add_argument("--max-iter", type=int, default=500)
    args = ap.parse_args()
    import torch
    hp = load_pkg()
    hp.set_device(0)
    M = hp.Matrix.generate(args.n, args.n, args.n, use_7pt=args.stencil == 7)
    b = M.vectors()[0]
    x = torch.zeros(args.n ** 3, dtype=torch.float64, device="cuda:0")
    variants = [parse(v) for v in args.variants.split(";")]
    keys = sorted({k for v in variants for k in v})
    # each key's value before any variant touches it (-1 is not valid for every option)
    defaults = {k: M.get_option(k) for k in keys}

    def apply(v):
        for k in keys:
            M.set_option(k, v.get(k, defaults[k]))

    def solve():
        x.zero_()
        return hp.HPCCG(M, b, x, max_iter=args.max_iter, device=True)[1]

    rates = [[] for _ in variants]
    ktimes = [None] * len(variants)
    traces = [None] * len(variants)
    for i, v in enumerate(variants):  # warm: graph capture, then one event-timed solve
        apply(v)
        solve()
        M.set_option("event_timing", 1)
        solve()
        kt = M.kernel_times()
        ktimes[i] = (kt["spmv_ms"] / kt["spmv_launches"] * 1e3, kt["update_ms"] / kt["update_launches"] * 1e3)
        M.set_option("event_timing", 0)
        traces[i] = M.last_trace().tobytes()
    for _ in range(args.reps):
        for i, v in enumerate(variants):
            apply(v)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.solves):
                it = solve()
            torch.cuda.synchronize()
            rates[i].append(it * args.solves / (time.perf_counter() - t0))
    for i, v in enumerate(variants):
        print(json.dumps({"n": args.n, "stencil": args.stencil, "options": v,
                          "it_per_s_median": round(statistics.median(rates[i]), 1),
                          "it_per_s_all": [round(r, 1) for r in rates[i]],
                          "spmv_us": round(ktimes[i][0], 2), "update_us": round(ktimes[i][1], 2),
                          "trace_equal_first": traces[i] == traces[0]}), flush=True)


if __name__ == "__main__":
    main()
