#!/usr/bin/env python3
"""The rate a caller of the reference's own interface sees (the host-pointer
boundary): HPCCG(A, b, x, ...) on a host
HPC_Sparse_Matrix through the C drop-in hpccg_hip_HPCCG (HPCCG.hpp:61-63) --
the device image cached per matrix, so a repeated call pays the content
fingerprint of A (host threads), the PCIe copies of b and x and the solve --
against the device-resident solve bench.py times (inputs already in HBM).

usage: python tools/host_rate.py [--n 200] [--stencil 27] [--solves 5]
Prints one JSON line per configuration."""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import load_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[200, 100])
    ap.add_argument("--stencil", type=int, default=27)
    ap.add_argument("--solves", type=int, default=5)
    ap.add_argument("--max-iter", type=int, default=500)
    args = ap.parse_args()
    import torch
    hp = load_pkg()
    hp.set_device(0)
    for n in args.n:
        s7 = args.stencil == 7
        t0 = time.perf_counter()
        prob = hp.generate_matrix(n, n, n, use_7pt=s7)
        gen_s = time.perf_counter() - t0
        out = {"n": n, "stencil": args.stencil, "host_generate_s": round(gen_s, 3)}
        # drop-in: first call builds and caches the device image. The C entry
        # point is called directly on prepared arrays (the Python wrapper's
        # copy of b would be timed otherwise)
        import ctypes as C
        L = hp.lib()
        bh = np.ascontiguousarray(prob.b)
        ni, nrm = C.c_int(0), C.c_double(0.0)
        times = np.zeros(7)

        def dropin(x):
            rc = L.hpccg_hip_HPCCG(prob.A, bh.ctypes.data, x.ctypes.data, args.max_iter, 0.0, C.byref(ni),
                                   C.byref(nrm), times.ctypes.data_as(C.POINTER(C.c_double)))
            hp._check(rc, "hpccg_hip_HPCCG")
            return ni.value

        x = prob.x
        t0 = time.perf_counter()
        dropin(x)
        out["dropin_first_call_s"] = round(time.perf_counter() - t0, 3)
        walls, t0s = [], []
        for _ in range(args.solves):
            x = prob.x
            t0 = time.perf_counter()
            it = dropin(x)
            walls.append(time.perf_counter() - t0)
            t0s.append(times[0])
        w = statistics.median(walls)
        out.update({"niters": it, "dropin_wall_s": round(w, 5), "dropin_times0_s": round(statistics.median(t0s), 5),
                    "dropin_it_per_s": round(it / w, 1),
                    "x_err": float(np.max(np.abs(x - 1.0)))})
        # the same matrix, device-resident vectors (what bench.py's value times)
        M = hp.Matrix.from_hpc(prob)
        b = torch.from_numpy(prob.b).cuda()
        xd = torch.zeros(n ** 3, dtype=torch.float64, device="cuda:0")
        hp.HPCCG(M, b, xd, max_iter=args.max_iter, device=True)
        dw = []
        for _ in range(args.solves):
            xd.zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _, it2, _, _ = hp.HPCCG(M, b, xd, max_iter=args.max_iter, device=True)
            torch.cuda.synchronize()
            dw.append(time.perf_counter() - t0)
        d = statistics.median(dw)
        out.update({"device_wall_s": round(d, 5), "device_it_per_s": round(it2 / d, 1),
                    "host_boundary_overhead_s": round(w - d, 5),
                    "host_boundary_overhead_frac": round((w - d) / w, 4)})
        # the host-pointer solve on the device matrix (PCIe copies, no fingerprint)
        hw = []
        for _ in range(args.solves):
            xh = prob.x
            t0 = time.perf_counter()
            _, it3, _, _ = hp.HPCCG(M, bh, xh, max_iter=args.max_iter)
            hw.append(time.perf_counter() - t0)
        h = statistics.median(hw)
        out.update({"host_ptr_wall_s": round(h, 5), "host_ptr_it_per_s": round(it3 / h, 1)})
        M.close()
        prob.close()  # (destroyMatrix releases the drop-in's cached device image)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
