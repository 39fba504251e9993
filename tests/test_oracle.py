"""Pin the CPU oracle (oracle/hpccg_oracle.c) to the reference.

Golden vectors come from the reference compiled from its own sources
(tests/golden/make_golden.py); out_10x10x10_150.txt is the reference's own
sample output (/root/reference/out.txt). With one thread the oracle must be
BITWISE equal to the reference serial build.
"""
import hashlib
import os

import numpy as np
import pytest

import oracle
from conftest import ROOT, check_trace, solve_case, unb64, unhex, RTRANS_RTOL_1GPU


def nnz_formula_27(nx, ny, nz):
    return (3 * nx - 2) * (3 * ny - 2) * (3 * nz - 2)


def nnz_formula_7(nx, ny, nz):
    return 7 * nx * ny * nz - 2 * (nx * ny + ny * nz + nx * nz)


def test_generator_matches_reference_csr(golden):
    g = golden["csr_4x3x2"]
    A = oracle.generate(4, 3, 2)
    assert A.row_ptr.tolist() == g["row_ptr"]
    assert A.cols.tolist() == g["cols"]
    assert A.vals.tolist() == g["vals"]
    assert A.b.tolist() == g["b"]
    assert A.x.tolist() == g["x"]
    assert A.xexact.tolist() == g["xexact"]
    # generate_matrix.cpp:226 stores the 27*n approximation, not the true nnz
    assert g["total_nnz_field"] == 27 * 24


@pytest.mark.parametrize("dims", [(4, 3, 2), (10, 10, 10), (20, 20, 20), (13, 7, 5), (1, 1, 1),
                                  (2, 1, 3)])
def test_kat4_nnz(dims):
    assert oracle.generate(*dims).nnz == nnz_formula_27(*dims)
    assert oracle.generate(*dims, use_7pt=True).nnz == nnz_formula_7(*dims)


def test_kat1_A_times_ones_is_b():
    for dims, s7 in [((20, 20, 20), False), ((13, 7, 5), False), ((16, 16, 16), True)]:
        A = oracle.generate(*dims, use_7pt=s7)
        y = oracle.sparsemv(A, np.ones(A.nrow))
        assert np.array_equal(y, A.b)


@pytest.mark.parametrize("dims,expect", [((10, 10, 10), 66688), ((20, 20, 20), 258728),
                                         ((100, 100, 100), 7007848)])
def test_kat2_initial_rtrans(dims, expect):
    if dims[0] == 100:
        # analytic: sum over rows of (28 - nnz_row)^2 with nnz_row = prod of per-axis counts
        def axis(n):
            c = np.full(n, 3)
            c[0] -= 1
            c[-1] -= 1
            return c
        cnt = (axis(dims[0])[None, None, :] * axis(dims[1])[None, :, None]
               * axis(dims[2])[:, None, None])
        assert int(((28 - cnt) ** 2).sum()) == expect
        return
    A = oracle.generate(*dims)
    res = oracle.hpccg(A, max_iter=1)
    assert res["trace"][0] ** 2 == pytest.approx(expect, rel=1e-15)
    r = A.b - oracle.sparsemv(A, A.x)
    assert oracle.ddot(r, r) == float(expect)


def test_kernels_bitwise_vs_reference(golden):
    k = golden["kernels_20x20x20"]
    A = oracle.generate(20, 20, 20)
    v, w = unb64(k["v_b64"]), unb64(k["w_b64"])
    assert np.array_equal(oracle.sparsemv(A, v), unb64(k["Av_b64"]))
    assert np.array_equal(oracle.sparsemv(A, A.b), unb64(k["Ab_b64"]))
    Av = unb64(k["Av_b64"])
    assert oracle.ddot(v, Av) == unhex(k["ddot"]["v.Av"])
    assert oracle.ddot(v, v) == unhex(k["ddot"]["v.v"])
    assert oracle.ddot(v, w) == unhex(k["ddot"]["v.w"])
    for key, val in k["waxpby"].items():
        a, b = (float(t) for t in key.split(","))
        assert np.array_equal(oracle.waxpby(a, v, b, w), unb64(val)), key


def _case_matrix(c):
    return oracle.generate(c["nx"], c["ny"], c["nz"] * c["ranks"], use_7pt=c["use_7pt"])


@pytest.mark.parametrize("name", ["27pt_20x20x20", "27pt_10x10x10", "27pt_13x7x5",
                                  "27pt_16x16x16_x8ranks", "27pt_8x8x8_x2ranks", "7pt_32x32x32",
                                  "7pt_12x10x8_x2ranks"])
def test_solve_bitwise_vs_reference(golden, name):
    c = solve_case(golden, name)
    A = _case_matrix(c)
    for mi, run in c["runs"].items():
        res = oracle.hpccg(A, max_iter=int(mi))
        assert res["niters"] == run["niters"]
        assert res["normr"] == unhex(run["normr"])
        assert hashlib.sha256(res["x"].tobytes()).hexdigest() == run["x_sha256"]
        if "x_b64" in run:
            assert np.array_equal(res["x"], unb64(run["x_b64"]), equal_nan=True)
    tr = [unhex(t) for t in c["trace_normr"]]
    res = oracle.hpccg(A, max_iter=len(tr))
    m = min(len(tr), res["niters"] + 1)
    assert np.array_equal(res["trace"][:m], np.array(tr[:m]))


def test_underflow_exit_10cubed(golden):
    """10^3 stops at niters=274 when rtrans underflows to 0 (HPCCG.cpp:358)."""
    c = solve_case(golden, "27pt_10x10x10")
    assert c["runs"]["500"]["niters"] == 274
    assert unhex(c["runs"]["500"]["normr"]) == 0.0


def test_reference_sample_output_out_txt():
    """/root/reference/out.txt: 10^3, 150 iterations. Its build is unknown, so
    only the lines before the residual reaches rounding noise are pinned."""
    lines = open(os.path.join(ROOT, "tests", "golden", "out_10x10x10_150.txt")).read().splitlines()
    A = oracle.generate(10, 10, 10)
    res = oracle.hpccg(A, max_iter=150)
    assert res["niters"] == 149
    assert lines[0] == "Initial Residual = %g" % res["trace"][0]
    assert lines[1] == "Iteration = 15   Residual = %g" % res["trace"][15]
    assert "Number of iterations: 149" in lines
    # FLOPS summary uses total_nnz = 27*n (main.cpp:222-226)
    n = 1000
    assert "  DDOT    : %g" % (149 * 4 * n) in lines
    assert "  WAXPBY  : %g" % (149 * 6 * n) in lines
    assert "  SPARSEMV: %g" % (149 * 2 * 27 * n) in lines


def test_openmp_within_stated_tolerance(golden):
    """Multithreaded oracle (nondeterministic combine order) stays inside the
    stated rtrans tolerance of the serial reference -- the envelope the GPU
    path is held to."""
    c = solve_case(golden, "27pt_20x20x20")
    A = _case_matrix(c)
    res = oracle.hpccg(A, max_iter=151, nthreads=4)
    tr = [unhex(t) for t in c["trace_normr"]]
    assert check_trace(res["trace"], tr, RTRANS_RTOL_1GPU) > 20


@pytest.mark.skipif(not oracle.ref_available(), reason="reference build only in the dev container")
def test_oracle_vs_live_reference_extra_sizes():
    for dims in [(9, 11, 7), (5, 5, 40)]:
        M, x0, b, xe = oracle.ref_generate(*dims)
        rp, cols, vals = M.to_csr()
        A = oracle.generate(*dims)
        assert np.array_equal(rp, A.row_ptr) and np.array_equal(cols, A.cols)
        assert np.array_equal(vals, A.vals) and np.array_equal(b, A.b)
        M.close()


@pytest.mark.skipif(not oracle.ref_available(), reason="reference build only in the dev container")
@pytest.mark.parametrize("nx,ny,nz,ranks", [(16, 16, 16, 8), (8, 8, 8, 2)])
def test_zstacked_goldens_matrix_is_the_reference_generators(nx, ny, nz, ranks):
    """The z-stacked goldens (27pt_16x16x16_x8ranks, 27pt_8x8x8_x2ranks) were
    solved by the reference on the oracle's global matrix. With MPI, rank r of
    the reference's generate_matrix builds global rows start_row = nx*ny*nz*r
    ... with global columns checked against total_nrow = nx*ny*nz*size
    (generate_matrix.cpp:225-266): exactly rows [start_row, stop_row] of the
    serial generate_matrix(nx, ny, nz*size). So the unmodified reference
    generator, run serially on the global dims, pins those matrices too: CSR,
    b, x and xexact bitwise, and every slab's columns stay within one plane of
    its rows (the z-slab halo exchange_externals moves)."""
    M, x0, b, xe = oracle.ref_generate(nx, ny, nz * ranks)
    rp, cols, vals = M.to_csr()
    A = oracle.generate(nx, ny, nz * ranks)
    assert np.array_equal(rp, A.row_ptr) and np.array_equal(cols, A.cols)
    assert np.array_equal(vals, A.vals) and np.array_equal(b, A.b)
    assert np.array_equal(x0, A.x) and np.array_equal(xe, A.xexact)
    M.close()
    n_loc, plane = nx * ny * nz, nx * ny
    for r in range(ranks):
        lo, hi = rp[r * n_loc], rp[(r + 1) * n_loc]
        c = cols[lo:hi]
        assert c.min() >= max(0, r * n_loc - plane) and c.max() < min(ranks * n_loc, (r + 1) * n_loc + plane)


@pytest.mark.skipif(not oracle.ref_available(), reason="reference build only in the dev container")
def test_reference_build_not_interposed_by_our_library(hp, golden):
    """Our libhpccg_hip.so exports the drop-in HPCCG() symbol; the reference
    build (linked -Bsymbolic, ours loaded RTLD_LOCAL) must still run its own
    CPU HPCCG -- with no GPU here, an interposed call would fail."""
    hp.lib()
    c = solve_case(golden, "27pt_10x10x10")
    M, x0, b, xe = oracle.ref_generate(10, 10, 10)
    import subprocess, sys
    res = oracle.ref_hpccg(M, b, max_iter=150)
    M.close()
    assert res["niters"] == c["runs"]["150"]["niters"]
    assert res["normr"] == unhex(c["runs"]["150"]["normr"])


@pytest.mark.skipif(not oracle.ref_available(), reason="reference build only in the dev container")
def test_degenerate_starts_match_reference():
    """Pins the oracle on the degenerate starts tests/test_gpu_edge.py checks
    the GPU against (HPCCG.cpp:347-386): a zero initial residual (no
    iteration), the 0/0 path under a negative tolerance (niters 2, NaN), NaN
    in b or x0 (no iteration), an infinite x0 entry on an interior row and on
    a face row (no iteration either: p = x + 0.0 x, HPCCG.cpp:347 through
    waxpby.cpp:77, is NaN there), and an infinite b entry (r0 = b - A x0 holds
    inf, r0.r0 = inf > 0: k = 1 forms p = r + 0.0 r, NaN, and the NaN path
    ends at niters 2). Same niters, normr bitwise or both NaN, x bitwise with
    NaN in the same places."""
    import math
    nx, ny, nz = 9, 11, 7
    M, _, b, _ = oracle.ref_generate(nx, ny, nz)
    A = oracle.generate(nx, ny, nz)
    n = A.nrow
    interior = (nz // 2) * nx * ny + (ny // 2) * nx + nx // 2
    face = (nz // 2) * nx * ny + (ny // 2) * nx + nx - 1  # the x = nx-1 face
    bn = b.copy()
    bn[n // 3] = np.nan
    xn = np.zeros(n)
    xn[n // 2 + 7] = np.nan
    xi = np.zeros(n)
    xi[interior] = np.inf
    xf = np.zeros(n)
    xf[face] = np.inf
    bi = b.copy()
    bi[face] = -np.inf
    todo = [("exact", b, np.ones(n), 30, 0.0, 0), ("zero_rhs", np.zeros(n), np.zeros(n), 30, 0.0, 0),
            ("exact_negtol", b, np.ones(n), 30, -1.0, 2), ("nan_b", bn, np.zeros(n), 30, 0.0, 0),
            ("nan_x0", b, xn, 30, 0.0, 0), ("inf_interior", b, xi, 30, 0.0, 0), ("inf_face", b, xf, 30, 0.0, 0),
            ("inf_b", bi, np.zeros(n), 30, 0.0, 2)]
    for name, bb, x0, mi, tol, want in todo:
        ref = oracle.ref_hpccg(M, bb, max_iter=mi, tolerance=tol, x=x0)
        got = oracle.hpccg(A, b=bb, x=x0, max_iter=mi, tolerance=tol)
        assert ref["niters"] == got["niters"] == want, name
        assert (math.isnan(ref["normr"]) and math.isnan(got["normr"])) or ref["normr"] == got["normr"], name
        assert np.array_equal(ref["x"], got["x"], equal_nan=True), name
    M.close()
