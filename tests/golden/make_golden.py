#!/usr/bin/env python3
"""Generate golden vectors from the REFERENCE compiled from its own sources.

Run here (where /root/reference exists) after ``make -C oracle ref``:

    python tests/golden/make_golden.py

Every number written below comes out of a reference function
(generate_matrix.cpp, HPC_sparsemv.cpp, ddot.cpp, waxpby.cpp, HPCCG.cpp, or the
reference test_HPCCG binary) via oracle/_ref -- never from our restatement.
The one exception is clearly marked: the 7-pt and z-stacked matrices are
*built* by the oracle generator (the unmodified reference generator hard-codes
27-pt and size=1, generate_matrix.cpp:210-219) and then *solved* by the
reference HPCCG(); tests/test_oracle.py separately pins that generator
against the reference one on the 27-pt serial case.

Per-iteration residual traces are obtained from the unmodified HPCCG() by a
max_iter sweep: the normr returned with max_iter=m is the normr computed in
iteration m-1 (HPCCG.cpp:358-373), and the initial residual for m=1.
"""
from __future__ import annotations

import base64
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


class quiet_stdout:
    """Silence fd 1 (the reference prints its residual lines with cout)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        self.null = os.open(os.devnull, os.O_WRONLY)
        os.dup2(self.null, 1)

    def __exit__(self, *a):
        import ctypes
        ctypes.CDLL(None).fflush(None)
        os.dup2(self.saved, 1)
        os.close(self.null)
        os.close(self.saved)


def b64(a: np.ndarray) -> str:
    return base64.b64encode(np.ascontiguousarray(a).tobytes()).decode()


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, np.float64).tobytes()).hexdigest()


def test_vector(n: int) -> np.ndarray:
    """Deterministic, libm-free vector: exact integer arithmetic then one division."""
    i = np.arange(n, dtype=np.int64)
    return (((i * 7919 + 13) % 1000) - 500).astype(np.float64) / 37.0


def sweep_trace(M, b, m_max, x0=None):
    """normr_trace[k] for k = 0..m_max-1 via max_iter = k+1 runs of HPCCG()."""
    tr = []
    with quiet_stdout():
        for m in range(1, m_max + 1):
            tr.append(oracle.ref_hpccg(M, b, max_iter=m, x=x0)["normr"])
    return tr


def solve_case(name, M, b, n, max_iters, sweep, store_x=False, extra=None, x0=None):
    case = {"name": name, "nrow": n, "runs": {}}
    if extra:
        case.update(extra)
    for mi in max_iters:
        with quiet_stdout():
            res = oracle.ref_hpccg(M, b, max_iter=mi, x=x0)
        x = res["x"]
        run = {
            "max_iter": mi,
            "niters": res["niters"],
            "normr": res["normr"].hex(),
            "x_minus_1_inf": float(np.max(np.abs(x - 1.0))) if np.all(np.isfinite(x)) else None,
            "x_sha256": sha(x),
            "x_finite": bool(np.all(np.isfinite(x))),
        }
        if store_x:
            run["x_b64"] = b64(x)
        case["runs"][str(mi)] = run
    if sweep:
        case["trace_normr"] = [v.hex() for v in sweep_trace(M, b, sweep, x0)]
    return case


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True,
                   stderr=subprocess.DEVNULL)
    assert oracle.ref_available()
    golden = {"source": "reference compiled from /root/reference (oracle/Makefile ref); "
                        "g++ -O3 -funroll-all-loops -malign-double -DWALL, serial"}

    # A. Exact CSR of a 4x3x2 grid from the reference generator.
    M, x0, b, xe = oracle.ref_generate(4, 3, 2)
    rp, cols, vals = M.to_csr()
    golden["csr_4x3x2"] = {"row_ptr": rp.tolist(), "cols": cols.tolist(),
                           "vals": vals.tolist(), "b": b.tolist(), "x": x0.tolist(),
                           "xexact": xe.tolist(), "total_nnz_field": oracle.ref_lib().ref_total_nnz(M.h)}
    M.close()

    # B. Kernel vectors on the 20^3 reference matrix.
    M, x0, b, xe = oracle.ref_generate(20, 20, 20)
    n = M.nrow
    v = test_vector(n)
    w = test_vector(n + 17)[17:] * 0.5 - 3.0
    L = oracle.ref_lib()
    y = np.zeros(n)
    L.ref_sparsemv(M.h, v, y)
    k = {"n": n, "v_b64": b64(v), "w_b64": b64(w), "Av_b64": b64(y),
         "Ab_sha256": None, "ddot": {}, "waxpby": {}}
    yb = np.zeros(n)
    L.ref_sparsemv(M.h, b, yb)
    k["Ab_b64"] = b64(yb)
    k["ddot"]["v.Av"] = L.ref_ddot(n, v, y).hex()
    k["ddot"]["v.v"] = L.ref_ddot(n, v, v).hex()
    k["ddot"]["v.w"] = L.ref_ddot(n, v, w).hex()
    for (a, bb) in [(1.0, 0.37), (2.5, 1.0), (-1.25, 0.75), (1.0, 0.0), (1.0, -1.0)]:
        out = np.zeros(n)
        L.ref_waxpby(n, a, v, bb, w, out)
        k["waxpby"][f"{a!r},{bb!r}"] = b64(out)
    golden["kernels_20x20x20"] = k

    # C. Solves (serial reference HPCCG).
    cases = []
    cases.append(solve_case("27pt_20x20x20", M, b, n, [150, 500], sweep=151, store_x=True,
                            extra={"nx": 20, "ny": 20, "nz": 20, "ranks": 1, "use_7pt": False}))
    M.close()
    M, x0, b, xe = oracle.ref_generate(10, 10, 10)
    cases.append(solve_case("27pt_10x10x10", M, b, M.nrow, [150, 500], sweep=300, store_x=True,
                            extra={"nx": 10, "ny": 10, "nz": 10, "ranks": 1, "use_7pt": False}))
    M.close()
    M, x0, b, xe = oracle.ref_generate(13, 7, 5)
    cases.append(solve_case("27pt_13x7x5", M, b, M.nrow, [500], sweep=120, store_x=True,
                            extra={"nx": 13, "ny": 7, "nz": 5, "ranks": 1, "use_7pt": False}))
    M.close()
    # Matrices built by the oracle generator (see module docstring), solved by the reference.
    for (nx, ny, nz, P, s7, sweep) in [(16, 16, 16, 8, False, 80), (8, 8, 8, 2, False, 100),
                                        (32, 32, 32, 1, True, 100), (12, 10, 8, 2, True, 100)]:
        A = oracle.generate(nx, ny, nz * P, use_7pt=s7)
        RM = oracle.ref_from_csr(A)
        name = f"{'7pt' if s7 else '27pt'}_{nx}x{ny}x{nz}" + (f"_x{P}ranks" if P > 1 else "")
        cases.append(solve_case(name, RM, A.b, A.nrow, [500], sweep=sweep,
                                extra={"nx": nx, "ny": ny, "nz": nz, "ranks": P, "use_7pt": s7,
                                       "matrix_from": "oracle generator (global nz*ranks)"}))
        RM.close()
    # Mode 2 (read_HPC_row.cpp) system: built by tests/golden/filemode.py (no RNG),
    # solved by the reference HPCCG() from the file's initial guess.
    sys.path.insert(0, OUT)
    import filemode
    rp, cl, vl, fx0, fb, fxe = filemode.general_system(600)
    RM = oracle.ref_from_csr(oracle.CSR(rp, cl, vl, fx0, fb, fxe))
    cases.append(solve_case("file_general_600", RM, fb, 600, [150, 500], sweep=120, x0=fx0,
                            extra={"ranks": 1, "matrix_from": "tests/golden/filemode.py general_system(600)"}))
    RM.close()
    golden["solves"] = cases

    # D. Reference CLI stdout (timings vary; tests compare structure and the
    #    deterministic lines).
    tmp = os.path.join("/tmp", "hpccg_golden_cli")
    os.makedirs(tmp, exist_ok=True)
    for dims in [(20, 20, 20), (10, 10, 10)]:
        out = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "test_HPCCG"), *map(str, dims)],
                             cwd=tmp, capture_output=True, text=True, check=True).stdout
        with open(os.path.join(OUT, "ref_cli_%dx%dx%d.txt" % dims), "w") as f:
            f.write(out)

    # Mode 2 through the reference CLI (its own read_HPC_row.cpp)
    fpath = os.path.join(tmp, "general_600.dat")
    filemode.write(fpath, rp, cl, vl, fx0, fb, fxe)
    out = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "test_HPCCG"), fpath],
                         cwd=tmp, capture_output=True, text=True, check=True).stdout
    with open(os.path.join(OUT, "ref_cli_file_general_600.txt"), "w") as f:
        f.write(out.replace(fpath, "<DATA_FILE>"))

    with open(os.path.join(OUT, "golden.json"), "w") as f:
        json.dump(golden, f, separators=(",", ":"))
    print("wrote", os.path.join(OUT, "golden.json"))


if __name__ == "__main__":
    main()
