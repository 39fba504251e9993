#!/usr/bin/env python3
"""Which buffer's physical placement moves the SpMV rate: for each buffer
class in turn, --rounds times move it to new memory (hpccg_hip_diag_realloc;
contents copied, the old one held) and time the CG iteration and the SpMV
launch. Diagnostics for the box-to-box / allocation-to-allocation spread.

With --probe: alternately create the matrix with the placement probe off
and on (hpccg_hip_probe_placement at creation), print the probe's per-
candidate SpMV times and the CG rate of each.

usage: tools/placement.py --n 200 --rounds 5
       tools/placement.py --n 200 --probe 6 --rounds 3
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import load_pkg  # noqa: E402

NAMES = {0: "values", 1: "p_ring", 2: "r", 3: "Ap", 4: "x"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--stencil", type=int, default=27)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--which", default="0,1,2,3")
    ap.add_argument("--mode", type=int, default=0, help="0 hipMalloc, 1 contiguous, 2/3/4 VMM 2 MB/64 MB/1 GB")
    ap.add_argument("--max-iter", type=int, default=200)
    ap.add_argument("--probe", default="0", help="candidates of the creation probe (A/B mode; a list "
                                                   "such as 6,10 alternates those counts after 0)")
    args = ap.parse_args()
    import torch
    hp = load_pkg()
    hp.set_device(0)
    if args.probe != "0":
        return probe_ab(hp, torch, args)
    hp.set_placement_probe(0)  # the creation placement as hipMalloc leaves it
    M = hp.Matrix.generate(args.n, args.n, args.n, use_7pt=args.stencil == 7)
    b = M.vectors()[0]
    x = torch.zeros(args.n ** 3, dtype=torch.float64, device="cuda:0")
    measure = make_measure(hp, torch, M, b, x, args.max_iter)
    r0, s0 = measure()
    print(json.dumps({"moved": None, "it_per_s": round(r0, 1), "spmv_us": round(s0, 2)}), flush=True)
    for w in [int(v) for v in args.which.split(",")]:
        for rnd in range(args.rounds):
            va = M.diag_realloc(w, args.mode)
            r, sp = measure()
            print(json.dumps({"moved": NAMES[w], "mode": args.mode, "round": rnd, "va_mod_1g_mb": (va % (1 << 30)) >> 20,
                              "it_per_s": round(r, 1), "spmv_us": round(sp, 2)}), flush=True)
    M.close()


def probe_ab(hp, torch, args):
    for rnd in range(args.rounds):
        for tries in [0] + [int(v) for v in args.probe.split(",")]:
            hp.set_placement_probe(tries)
            t0 = time.perf_counter()
            M = hp.Matrix.generate(args.n, args.n, args.n, use_7pt=args.stencil == 7)
            setup_s = time.perf_counter() - t0
            b = M.vectors()[0]
            x = torch.zeros(args.n ** 3, dtype=torch.float64, device="cuda:0")
            r, sp = make_measure(hp, torch, M, b, x, args.max_iter)()
            print(json.dumps({"round": rnd, "probe": tries, "setup_s": round(setup_s, 3),
                              "probe_us": [round(float(v), 2) for v in M.placement()],
                              "pick": [(M.get_option("placement_pick") >> (8 * i)) & 255 for i in range(4)], "it_per_s": round(r, 1),
                              "spmv_us": round(sp, 2)}), flush=True)
            M.close()
            del b, x
    hp.set_placement_probe(-1)


def make_measure(hp, torch, M, b, x, max_iter):
    args = argparse.Namespace(max_iter=max_iter)

    def measure():
        x.zero_()
        hp.HPCCG(M, b, x, max_iter=args.max_iter, device=True)  # capture
        M.set_option("event_timing", 1)
        x.zero_()
        hp.HPCCG(M, b, x, max_iter=args.max_iter, device=True)
        kt = M.kernel_times()
        M.set_option("event_timing", 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x.zero_()
        it = hp.HPCCG(M, b, x, max_iter=args.max_iter, device=True)[1]
        torch.cuda.synchronize()
        return it / (time.perf_counter() - t0), kt["spmv_ms"] / kt["spmv_launches"] * 1e3
    return measure


if __name__ == "__main__":
    main()
