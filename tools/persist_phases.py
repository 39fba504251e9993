#!/usr/bin/env python3
"""Phases of the persistent CG launch from the device stamps (block 0 and the
top waiters): per iteration, SPARSEMV = slot loop + p.Ap partials
+ group/top completion, DDOT = the broadcast to block 0 (both dots), WAXPBY =
the update + r.r partials + completion. usage: tools/persist_phases.py [--n 100]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import load_pkg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=100)
ap.add_argument("--shapes", default="1,-1", help="resident_update values (1 k_spmv_ar, -1 the persistent launch)")
args = ap.parse_args()
import torch  # noqa: E402
hp = load_pkg()
hp.set_device(0)
M = hp.Matrix.generate(args.n, args.n, args.n)
b, _, _ = M.vectors()
x = torch.zeros(args.n ** 3, dtype=torch.float64, device="cuda:0")
names = ["total", "ddot", "waxpby", "sparsemv", "allreduce", "halo", "?"]
for shape in [int(v) for v in args.shapes.split(",")]:
    M.set_option("resident_update", shape)
    for rep in range(3):
        x.zero_()
        _, it, _, t = hp.HPCCG(M, b, x, max_iter=500, device=True)
    print(f"resident_update {shape} ({M.get_option('resident_update')}): " +
          ", ".join(f"{nm} {t[i] / it * 1e6:.2f} us/it" for i, nm in enumerate(names[:4])), flush=True)
