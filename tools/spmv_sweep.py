#!/usr/bin/env python3
"""Sweep SpMV kernel variants on the device-generated stencil matrix.

Times each variant with hipEvents (hpccg_hip_diag_spmv: back-to-back launches
on the solver stream) and reports algorithmic GB/s = (12 nnz + 20 n) / time.
Variant 9999 is the matrix-streaming ceiling (no x gather; not an SpMV).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import load_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[200, 100])
    ap.add_argument("--stencil", type=int, default=27)
    ap.add_argument("--variants", type=int, nargs="+",
                    default=[1000, 1001, 2000, 2001, 2002, 2100, 9999, 1000, 2000])
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch  # noqa: F401
    hp = load_pkg()
    hp.set_device(0)
    for n in args.n:
        M = hp.Matrix.generate(n, n, n, use_7pt=args.stencil == 7)
        info = M.info()
        nbytes = 12.0 * info["nnz"] + 20.0 * info["nrow"]
        for v in args.variants:
            try:
                us = M.diag_spmv(v, args.reps)
            except Exception as e:  # variant not valid for this matrix
                print(json.dumps({"n": n, "variant": v, "error": str(e)}), flush=True)
                continue
            print(json.dumps({"n": n, "stencil": args.stencil, "variant": v, "us": round(us, 2),
                              "GBs": round(nbytes / us / 1e3, 1),
                              "frac": round(nbytes / us / 1e3 / 8000, 4)}), flush=True)
        M.close()


if __name__ == "__main__":
    main()
