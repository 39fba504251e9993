#!/usr/bin/env python3
"""Per-iteration SpMV / update launch times of one event-timed solve, grouped
by the p ring slot (k % x_ring): tells whether the launch time depends on which
buffers an iteration streams (placement) rather than on the iteration.

usage: tools/iter_times.py --n 256 --stencil 7
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import load_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--stencil", type=int, default=27)
    ap.add_argument("--solves", type=int, default=2)
    args = ap.parse_args()
    import torch
    hp = load_pkg()
    hp.set_device(0)
    M = hp.Matrix.generate(args.n, args.n, args.n, use_7pt=args.stencil == 7)
    b = M.vectors()[0]
    x = torch.zeros(args.n ** 3, dtype=torch.float64, device="cuda:0")
    ring = M.get_option("x_ring")
    M.set_option("event_timing", 1)
    for s in range(args.solves):
        x.zero_()
        hp.HPCCG(M, b, x, max_iter=500, device=True)
        t = M.kernel_times_iter() * 1e3  # us
        k = np.arange(len(t))
        by = {}
        for slot in range(ring):
            sel = (k % ring == slot) & (k > 0)
            by[slot] = [round(float(np.median(t[sel, 0])), 1), round(float(np.median(t[sel, 1])), 1)]
        print(json.dumps({"solve": s, "ring": ring, "spmv_us_median": round(float(np.median(t[1:, 0])), 2),
                          "spmv_us_min": round(float(t[1:, 0].min()), 2), "spmv_us_max": round(float(t[1:, 0].max()), 2),
                          "by_ring_slot_spmv_update_us": by,
                          "first_40_spmv_us": [round(float(v), 1) for v in t[1:41, 0]]}), flush=True)


if __name__ == "__main__":
    main()
