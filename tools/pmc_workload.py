#!/usr/bin/env python3
"""Workload for the rocprofv3 --pmc passes: the known-bytes stream of the
SELL-512-A values (FETCH_SIZE calibration, hpccg_hip_diag_spmv kernel 9) and a
short eager CG solve with the production kernels."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import load_pkg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=200)
ap.add_argument("--iters", type=int, default=32)  # x_defer 2: every launch but the first carries side blocks
ap.add_argument("--stencil", type=int, default=27, choices=[27, 7])
ap.add_argument("--kernel", type=int, default=-1, help="SpMV kernel (-1: the library's choice)")
ap.add_argument("--fuse-p", type=int, default=-1, help="p update inside the SpMV (-1: default)")
args = ap.parse_args()
import torch  # noqa: E402,F401
hp = load_pkg()
hp.set_device(0)
M = hp.Matrix.generate(args.n, args.n, args.n, use_7pt=args.stencil == 7)
M.diag_spmv(9, 3)  # known-bytes stream of the A image (FETCH calibration)
if args.kernel >= 0:
    M.set_option("spmv_kernel", args.kernel)
if args.fuse_p >= 0:
    M.set_option("fuse_p", args.fuse_p)
b, _, _ = M.vectors()
x = torch.zeros(args.n ** 3, dtype=torch.float64, device="cuda:0")
M.set_option("use_graph", 0)
hp.HPCCG(M, b, x, max_iter=args.iters, device=True)
print("fuse_p", M.get_option("fuse_p"), "kernel", M.get_option("spmv_kernel"), "slots", M.info()["slots"],
      "x_defer", M.get_option("x_defer"), "x_ring", M.get_option("x_ring"))
