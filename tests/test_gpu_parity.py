"""Parity of the MI355X HIP path against the oracle and the reference goldens.

All calls go through the C ABI (libhpccg_hip.so). Bars:
* HPC_sparsemv and waxpby: BITWISE equal to the reference (same entry order,
  no FMA contraction);
* ddot: deterministic (bitwise run to run) and within 1e-13 relative of the
  reference's sequential sum (different association only);
* HPCCG: niters equal; rtrans_k within RTRANS_RTOL_1GPU = 1e-8 relative for
  every k with rtrans_ref,k >= 1e-20 * rtrans_ref,0; final relative residual
  <= 1e-15 (or underflow to 0 exactly where the reference underflows);
  |x - 1|_inf <= 1e-12.
Every SpMV kernel (SELL-512, SELL-512-A direct, SELL-512-A pair windows), the
fused p update, the dot folding, graph replay and the x deferral change where
work happens, never a value: the tests below require bitwise equal solves.
"""
import itertools
import math
import os

import numpy as np
import pytest

import oracle
from conftest import (RTRANS_RTOL_1GPU, check_final, check_trace, kat2_rr0, solve_case, unb64, unhex)

pytestmark = pytest.mark.gpu

DDOT_RTOL = 1e-13
SELL, DIRECT, PAIRS = 0, 1, 2


def dev(torch_device, a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, np.float64)).to(torch_device)


def host(t):
    return t.cpu().numpy()


@pytest.fixture
def keep_sell(hp):
    """Matrices created inside the test keep SELL-512 beside SELL-512-A, so the
    three kernels can be compared on one matrix."""
    hp.set_keep_sell(True)
    yield
    hp.set_keep_sell(False)


def solve_bits(hp, M, b, max_iter, gpu=None):
    """(niters, normr, trace bytes, x bytes) of one solve from x0 = 0."""
    if gpu is None:
        x = np.zeros(len(b))
        _, it, nr, _ = hp.HPCCG(M, b, x, max_iter=max_iter)
        return it, nr, M.last_trace().tobytes(), x.tobytes()
    import torch
    n = M.info()["nrow"]
    x = torch.zeros(n, dtype=torch.float64, device=gpu)
    _, it, nr, _ = hp.HPCCG(M, b, x, max_iter=max_iter, device=True)
    return it, nr, M.last_trace().tobytes(), host(x).tobytes()


# ---------------------------------------------------------------------------
# kernel level
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("kernel", [SELL, DIRECT])
def test_sparsemv_bitwise_vs_reference(hp, gpu, golden, keep_sell, kernel):
    import torch
    k = golden["kernels_20x20x20"]
    prob = hp.generate_matrix(20, 20, 20)
    M = hp.Matrix.from_hpc(prob)
    M.set_option("spmv_kernel", kernel)
    v = dev(gpu, unb64(k["v_b64"]))
    y = torch.zeros_like(v)
    hp.HPC_sparsemv(M, v, y)
    assert np.array_equal(host(y), unb64(k["Av_b64"]))
    bb = dev(gpu, prob.b)
    hp.HPC_sparsemv(M, bb, y)
    assert np.array_equal(host(y), unb64(k["Ab_b64"]))
    # KAT-1: A * 1 == b bitwise
    hp.HPC_sparsemv(M, torch.ones_like(v), y)
    assert np.array_equal(host(y), prob.b)


@pytest.mark.parametrize("dims,s7", [((24, 20, 18), False), ((13, 7, 5), False), ((40, 40, 40), False),
                                     ((32, 16, 40), True), ((17, 9, 11), True),
                                     # pair windows past one staging round of the ring kernel (3 x 1866 > 5120)
                                     ((420, 8, 24), False)])
def test_kernels_agree_bitwise(hp, gpu, keep_sell, dims, s7):
    """SELL-512 gather, SELL-512-A direct and SELL-512-A pair windows, with the
    p update separate or formed inside the SpMV, give bitwise the same solve
    (same row sums, same p.Ap tree)."""
    prob = hp.generate_matrix(*dims, use_7pt=s7)
    M = hp.Matrix.from_hpc(prob)
    assert M.get_option("has_a") == 1 and M.get_option("has_pairs") == 1 and M.get_option("has_sell") == 1
    assert M.get_option("a_width") == (7 if s7 else 27)
    out = {}
    for kernel, fuse in itertools.product((SELL, DIRECT, PAIRS), (0, -1)):
        M.set_option("spmv_kernel", kernel)
        M.set_option("fuse_p", fuse)
        assert M.get_option("spmv_kernel") == kernel
        assert M.get_option("fuse_p") == (1 if (fuse and kernel != SELL) else 0)
        out[(kernel, fuse)] = solve_bits(hp, M, prob.b, 120)
    # the pair kernel's value stream: register loads (0) or the LDS-DMA ring
    # (uniform widths 27 and 7); other ring depths are refused
    M.set_option("spmv_kernel", PAIRS)
    for fuse, ring in itertools.product((0, -1), (-1, 0, 3)):
        M.set_option("fuse_p", fuse)
        M.set_option("a2_ring", ring)
        assert M.get_option("a2_ring") == (3 if ring < 0 else ring)
        out[("ring", fuse, ring)] = solve_bits(hp, M, prob.b, 120)
    for ring in (1, 2, 4):
        with pytest.raises(hp.HPCCGError):
            M.set_option("a2_ring", ring)
    # x_defer 2: the deferred x terms applied by trailing blocks of the ring
    # kernel's launch (119 iterations: a different remainder per slice for k_xflush)
    for fuse, xring, graph in ((-1, 32, 1), (0, 32, 0), (-1, 2, 1), (-1, 5, 0), (0, 9, 1)):
        M.set_option("fuse_p", fuse)
        M.set_option("a2_ring", -1)
        M.set_option("x_defer", 2)
        M.set_option("x_ring", xring)
        M.set_option("use_graph", graph)
        assert M.get_option("x_defer") == 2
        out[("side", fuse, xring, graph)] = solve_bits(hp, M, prob.b, 120)
    M.set_option("a2_ring", 0)
    assert M.get_option("x_defer") == 1  # register-load pair kernel: batched in the update
    M.set_option("a2_ring", -1)
    # and by trailing blocks of the direct kernel's launch
    M.set_option("spmv_kernel", DIRECT)
    for fuse, xring in ((-1, 32), (0, 8), (-1, 3)):
        M.set_option("fuse_p", fuse)
        M.set_option("x_ring", xring)
        assert M.get_option("x_defer") == 2
        out[("side-direct", fuse, xring)] = solve_bits(hp, M, prob.b, 120)
    # the update as trailing blocks of the direct kernel's launch (fused update)
    M.set_option("x_ring", -1)
    for graph, chunk in ((1, 32), (0, 8), (1, 7), (1, 3), (0, 32)):
        M.set_option("fuse_p", -1)
        M.set_option("fold", 1)
        M.set_option("use_graph", graph)
        M.set_option("graph_chunk", chunk)
        M.set_option("fuse_update", 1)
        assert M.get_option("fuse_update") == 1
        out[("fused-update", graph, chunk)] = solve_bits(hp, M, prob.b, 120)
    M.set_option("fuse_update", 0)
    M.set_option("graph_chunk", 32)
    M.set_option("spmv_kernel", SELL)
    assert M.get_option("x_defer") == 1
    M.set_option("x_defer", 1)
    M.set_option("use_graph", 1)
    bad = [k for k, o in out.items() if o != out[(SELL, 0)]]
    assert not bad, bad


@pytest.mark.parametrize("dims", [(24, 20, 18), (13, 7, 5), (40, 40, 40)])
def test_fusion_options_bitwise_equal(hp, gpu, dims):
    """fuse_p, fold (last-block dot completion), graph replay, x_defer and the
    update's slice order change only where work happens, never a value: every
    combination gives bitwise the same solve, with the default kernel."""
    prob = hp.generate_matrix(*dims)
    M = hp.Matrix.from_hpc(prob)
    results = []
    # the persistent launch (auto where it fits) first; the per-iteration
    # launches these options shape below
    M.set_option("spmv_kernel", DIRECT)
    results.append(solve_bits(hp, M, prob.b, 120))
    M.set_option("resident_update", 0)
    for kernel in (DIRECT, PAIRS):
        M.set_option("spmv_kernel", kernel)
        for fuse, fold, graph, defer in itertools.product((0, -1), (0, 1), (0, 1), (0, 1, 2)):
            M.set_option("fuse_p", fuse)
            M.set_option("fold", fold)
            M.set_option("use_graph", graph)
            M.set_option("x_defer", defer)
            assert M.get_option("fold") == fold
            # 119 iterations: x updates left for k_xflush
            results.append(solve_bits(hp, M, prob.b, 120))
            if graph:
                assert M.get_option("graph_used") == 1
    # the x-deferral depth (p ring length) only moves when x is written:
    # rings of 2 .. 64, 119 iterations leave 1 .. 55 updates for k_xflush
    # (staggered: a different remainder per slice)
    M.set_option("fold", -1)
    for i, (ring, graph) in enumerate(((2, 1), (5, 0), (16, 1), (32, 1), (64, 0), (8, 1), (-1, 1), (32, 0), (5, 1))):
        M.set_option("x_defer", 1 + i % 2)
        M.set_option("x_ring", ring)
        M.set_option("use_graph", graph)
        assert M.get_option("x_ring") == (ring if ring > 0 else 8)  # auto: 8 for a small image
        results.append(solve_bits(hp, M, prob.b, 120))
    # graph chunks that do not divide the iteration count (eager tail)
    for chunk in (1, 3, 13, 64):
        M.set_option("graph_chunk", chunk)
        results.append(solve_bits(hp, M, prob.b, 120))
    assert all(r == results[0] for r in results)


@pytest.mark.parametrize("dims,reps", [((64, 64, 48), 12), ((96, 96, 100), 4)])
def test_folded_dot_completion_stress(hp, gpu, dims, reps):
    """The in-kernel (fold) dot completion hands partials between workgroups on
    different XCDs (self-validating slots). Any stale read would change a sum:
    repeat many solves and compare
    every trace bitwise with the separate k_finalize path (data handed over by
    a kernel boundary). 96x96x100: 1800 slices, 29 groups that straddle the
    XCD eighths of the grid (the waiting member is then not the group's last
    slice)."""
    prob = hp.generate_matrix(*dims)
    M = hp.Matrix.from_hpc(prob)
    for kernel in (DIRECT, PAIRS):
        M.set_option("spmv_kernel", kernel)
        M.set_option("fold", 0)
        ref = solve_bits(hp, M, prob.b, 150)
        for fold in (1, -1):
            M.set_option("fold", fold)
            for graph in (1, 0):
                M.set_option("use_graph", graph)
                for _ in range(reps):
                    assert solve_bits(hp, M, prob.b, 150) == ref, (kernel, fold, graph)


def test_waxpby_bitwise_vs_reference(hp, gpu, golden):
    import torch
    k = golden["kernels_20x20x20"]
    v, w = dev(gpu, unb64(k["v_b64"])), dev(gpu, unb64(k["w_b64"]))
    n = v.numel()
    for key, val in k["waxpby"].items():
        a, b = (float(t) for t in key.split(","))
        out = torch.zeros_like(v)
        hp.waxpby(n, a, v, b, w, out)
        assert np.array_equal(host(out), unb64(val)), key
    # in place (w aliases x), as HPCCG.cpp:369 / 383-384 use it
    x = v.clone()
    hp.waxpby(n, 1.0, x, 0.37, w, x)
    assert np.array_equal(host(x), unb64(k["waxpby"]["1.0,0.37"]))


def test_ddot_deterministic_and_close(hp, gpu, golden):
    k = golden["kernels_20x20x20"]
    v, w, Av = (dev(gpu, unb64(k[f])) for f in ("v_b64", "w_b64", "Av_b64"))
    n = v.numel()
    for name, (a, b) in {"v.Av": (v, Av), "v.v": (v, v), "v.w": (v, w)}.items():
        r1 = hp.ddot(n, a, b)
        r2 = hp.ddot(n, a, b)
        assert r1 == r2
        ref = unhex(k["ddot"][name])
        assert abs(r1 - ref) <= DDOT_RTOL * abs(ref), (name, r1, ref)


def test_ddot_edge_sizes(hp, gpu):
    import torch
    for n in [0, 1, 2, 63, 64, 65, 511, 512, 513, 4095, 4096, 4097, 100003]:
        a = np.arange(n, dtype=np.float64) % 7 - 3.0
        b = np.arange(n, dtype=np.float64) % 5 - 2.0
        r = hp.ddot(n, dev(gpu, a) if n else torch.zeros(1, dtype=torch.float64, device=gpu),
                    dev(gpu, b) if n else torch.zeros(1, dtype=torch.float64, device=gpu))
        assert r == float(np.dot(a, b)), n  # small integers: exact in any order


# ---------------------------------------------------------------------------
# full solves vs the reference goldens
# ---------------------------------------------------------------------------
def _matrix_for_case(hp, c, how):
    P = c["ranks"]
    if how == "device":
        return hp.Matrix.generate(c["nx"], c["ny"], c["nz"] * P, use_7pt=c["use_7pt"]), None
    prob = hp.generate_matrix(c["nx"], c["ny"], c["nz"] * P, use_7pt=c["use_7pt"])
    return hp.Matrix.from_hpc(prob), prob


@pytest.mark.parametrize("name", ["27pt_20x20x20", "27pt_10x10x10", "27pt_13x7x5",
                                  "27pt_16x16x16_x8ranks", "27pt_8x8x8_x2ranks", "7pt_32x32x32",
                                  "7pt_12x10x8_x2ranks"])
@pytest.mark.parametrize("how", ["host", "device"])
def test_solve_vs_reference(hp, gpu, golden, name, how):
    import torch
    c = solve_case(golden, name)
    M, prob = _matrix_for_case(hp, c, how)
    n = c["nrow"]
    ref_tr = [unhex(t) for t in c["trace_normr"]]

    def run(max_iter):
        if how == "host":
            x = prob.x
            _, it, nr, times = hp.HPCCG(M, prob.b, x, max_iter=max_iter)
            return it, nr, times, x
        b, _, _ = M.vectors()
        xt = torch.zeros(n, dtype=torch.float64, device=gpu)
        _, it, nr, times = hp.HPCCG(M, b, xt, max_iter=max_iter, device=True)
        return it, nr, times, host(xt)

    # the per-iteration trajectory (pre-convergence: 1e-8 on rtrans)
    it, nr, _, _ = run(len(ref_tr))
    tr = M.last_trace()
    assert tr[0] == ref_tr[0]  # KAT-2: integer-valued rtrans_0, exact in any order
    assert tr[1] == ref_tr[1]  # normr after iteration 1 is sqrt(rtrans_0) (HPCCG.cpp:371)
    # KAT-3: p = r_0 and A p are integer-valued, alpha_1 a correctly rounded quotient, so
    # r_1 matches elementwise and r_1.r_1 (a sum of n positive terms) differs only by the
    # summation order: the reference's serial sum is within (n-1) u of the exact value
    assert abs(tr[2] ** 2 - ref_tr[2] ** 2) <= 2 * n * 2.0 ** -53 * ref_tr[2] ** 2
    assert check_trace(tr, ref_tr, RTRANS_RTOL_1GPU) >= 5
    for mi, rr in c["runs"].items():
        it, nr, times, x = run(int(mi))
        tr = M.last_trace()
        assert len(tr) == it + 1
        check_final(it, nr, tr, rr["niters"], unhex(rr["normr"]), ref_tr, int(mi))
        if rr["x_finite"]:
            assert np.all(np.isfinite(x))
            assert np.max(np.abs(x - 1.0)) <= 1e-12
        assert times[0] > 0
        # the timer classes (device stamps) partition the solve
        assert 0.0 <= times[1] + times[2] + times[3] <= times[0] * 1.05 + 1e-3


def test_solve_reproducible(hp, gpu):
    prob = hp.generate_matrix(30, 30, 30)
    M = hp.Matrix.from_hpc(prob)
    assert solve_bits(hp, M, prob.b, 200) == solve_bits(hp, M, prob.b, 200)


def test_device_generator_matches_host(hp, gpu):
    """the device generator writes the same image."""
    import torch
    for dims, s7 in [((20, 20, 20), False), ((13, 7, 5), False), ((17, 9, 11), True)]:
        prob = hp.generate_matrix(*dims, use_7pt=s7)
        Mh = hp.Matrix.from_hpc(prob)
        Md = hp.Matrix.generate(*dims, use_7pt=s7)
        assert Mh.info() == Md.info()
        b, x0, xe = Md.vectors()
        n = prob.nrow
        bt = torch.empty(n, dtype=torch.float64, device=gpu)
        torch.cuda.synchronize()
        hp.waxpby(n, 1.0, b, 0.0, b, bt)  # copy device b through w = b + 0*b
        assert np.array_equal(host(bt), prob.b)
        x1 = prob.x
        hp.HPCCG(Mh, prob.b, x1, max_iter=80)
        t1 = Mh.last_trace()
        xt = torch.zeros(n, dtype=torch.float64, device=gpu)
        hp.HPCCG(Md, b, xt, max_iter=80, device=True)
        assert np.array_equal(t1, Md.last_trace())
        assert np.array_equal(x1, host(xt))


def test_edge_max_iter_and_tolerance(hp, gpu):
    prob = hp.generate_matrix(9, 8, 7)
    A = oracle.generate(9, 8, 7)
    M = hp.Matrix.from_hpc(prob)
    for mi in [0, 1, 2, 3, 9, 10]:
        x = prob.x
        _, it, nr, _ = hp.HPCCG(M, prob.b, x, max_iter=mi)
        ref = oracle.hpccg(A, max_iter=mi)
        assert it == ref["niters"], mi
        assert nr == pytest.approx(ref["normr"], rel=1e-10), mi
    # positive tolerance: stops where the oracle stops
    for tol in [1e-3, 1e-8, 1e-20]:
        x = prob.x
        _, it, nr, _ = hp.HPCCG(M, prob.b, x, max_iter=500, tolerance=tol)
        ref = oracle.hpccg(A, max_iter=500, tolerance=tol)
        assert it == ref["niters"], tol


def _random_sym(n, seed, kmax=40):
    """A general (non-stencil) SPD matrix with ragged row lengths: many
    distinct offsets per slice, so no SELL-512-A image."""
    rng = np.random.default_rng(seed)
    import collections
    nb = collections.defaultdict(set)
    for i in range(n):
        k = int(rng.integers(0, kmax))
        for c in np.unique(rng.integers(0, n, size=k)):
            if c != i:
                nb[i].add(int(c))
                nb[int(c)].add(i)
    row_ptr = [0]
    cols, vals = [], []
    for i in range(n):
        cs = sorted(nb[i] | {i})
        for c in cs:
            cols.append(c)
            vals.append(float(len(cs) + 1) if c == i else -1.0)
        row_ptr.append(len(cols))
    return np.array(row_ptr, np.int64), np.array(cols, np.int32), np.array(vals, np.float64)


def test_csr_entry_and_ragged_rows(hp, gpu):
    """A general SPD matrix with ragged row lengths through the CSR entry
    point: more than 32 offsets per slice, so the SELL-512 kernel runs and the
    A kernels are refused."""
    n = 1500
    row_ptr, cols, vals = _random_sym(n, 7)
    b = np.arange(n, dtype=np.float64) % 13 - 6.0
    A = oracle.CSR(row_ptr, cols, vals, np.zeros(n), b, np.ones(n))
    M = hp.Matrix.from_csr(row_ptr, cols, vals)
    assert M.get_option("has_a") == 0 and M.get_option("spmv_kernel") == SELL
    with pytest.raises(hp.HPCCGError, match="not built"):
        M.set_option("spmv_kernel", DIRECT)
    x = np.zeros(n)
    _, it, nr, _ = hp.HPCCG(M, b, x, max_iter=120)
    ref = oracle.hpccg(A, max_iter=120)
    assert it == ref["niters"]
    assert check_trace(M.last_trace(), ref["trace"], RTRANS_RTOL_1GPU) >= 5
    import torch
    v = (np.arange(n) % 17) / 3.0
    y = torch.zeros(n, dtype=torch.float64, device=gpu)
    hp.HPC_sparsemv(M, dev(gpu, v), y)
    assert np.array_equal(host(y), oracle.sparsemv(A, v))


# ---------------------------------------------------------------------------
# BASELINE sizes: full-size parity (oracle trace where it finishes in seconds)
# and size-independent properties
# ---------------------------------------------------------------------------
def _oracle_trace(dims, s7, iters):
    """The first `iters` iterations on the same matrix: the C restatement's
    full trace (OpenMP), and -- where oracle/_ref is built -- the unmodified
    reference HPCCG() (its OpenMP build, main.cpp's flags) at sampled
    iterations k, by max_iter = k + 1 runs (the normr it returns is the one
    computed in iteration k, HPCCG.cpp:358-373). Returns (trace, {k: normr}
    or None)."""
    A = oracle.generate(*dims, use_7pt=s7)
    tr = oracle.hpccg(A, max_iter=iters + 1, nthreads=max(1, min(16, oracle.max_threads())))["trace"]
    pts = None
    if os.path.exists(oracle.REF_OMP_SO):
        ks = sorted({k for k in (0, 1, 2, 3, 5, 8, 13, 21, 34, iters // 2, iters - 1) if 0 <= k < iters})
        M = oracle.ref_from_csr(A, omp=True)
        pts = {}
        saved, null = os.dup(1), os.open(os.devnull, os.O_WRONLY)
        os.dup2(null, 1)  # the reference prints its residual lines on fd 1
        try:
            for k in ks:
                pts[k] = oracle.ref_hpccg(M, A.b, max_iter=k + 1)["normr"]
        finally:
            import ctypes
            ctypes.CDLL(None).fflush(None)
            os.dup2(saved, 1)
            os.close(null)
            os.close(saved)
            M.close()
    del A
    return tr, pts


@pytest.mark.parametrize("dims,s7,trace_iters", [((100, 100, 100), False, 90),
                                                  ((200, 200, 200), False, 60),
                                                  ((256, 256, 256), True, 60),
                                                  ((320, 320, 320), False, 0),
                                                  ((432, 432, 432), False, 0)])
def test_full_size(hp, gpu, dims, s7, trace_iters, record_property):
    """BASELINE sizes (and 320^3: 32.8 M rows, 0.88 G nonzeros; 432^3: 80.6 M
    rows, 2.167 G nonzeros and 2.18 G A-image slots, past 2^31 -- every slot and
    nonzero count and offset 64-bit) on the default
    kernel: the first iterations' rtrans against the oracle on the same matrix
    (1e-8) -- the unmodified reference build (oracle/_ref) at sampled
    iterations where it is present, and the C restatement's full trace --,
    KAT-1 (A*1 == b bitwise), KAT-2 (rtrans_0 exact), KAT-4 (nnz formula), the
    full 499-iteration solve's final residual and x, and the device footprint
    (SELL-512 freed once the A image exists)."""
    import torch
    M = hp.Matrix.generate(*dims, use_7pt=s7)
    info = M.info()
    nx, ny, nz = dims
    n = nx * ny * nz
    if s7:
        assert info["nnz"] == 7 * n - 2 * (ny * nz + nx * nz + nx * ny)  # KAT-4
    else:
        assert info["nnz"] == (3 * nx - 2) * (3 * ny - 2) * (3 * nz - 2)  # KAT-4
    assert M.get_option("has_a") == 1 and M.get_option("has_sell") == 0
    # 8 B per slot of the A image, the p ring, r / Ap / x / b and the generated
    # b / x0 / xexact, and small tables (no SELL-512 image left)
    ring = M.get_option("x_ring")
    limit = info["slots"] * 8 + (ring + 7) * (n + 4 * 2048 + 2 * nx * ny) * 8 + 64e6
    assert M.get_option("device_bytes") <= limit
    if dims == (200, 200, 200):
        assert M.get_option("device_bytes") <= 4.5e9  # <= 4.5 GB per 200^3 rank
    b, x0, xe = M.vectors()
    ones = torch.ones(n, dtype=torch.float64, device=gpu)
    y = torch.empty(n, dtype=torch.float64, device=gpu)
    hp.HPC_sparsemv(M, ones, y)
    bt = torch.empty(n, dtype=torch.float64, device=gpu)
    hp.waxpby(n, 1.0, b, 0.0, b, bt)
    assert torch.equal(y, bt)  # KAT-1
    del ones, y, bt
    x = torch.zeros(n, dtype=torch.float64, device=gpu)
    _, it, nr, times = hp.HPCCG(M, b, x, max_iter=500, device=True)
    tr = M.last_trace()
    assert it == 499
    assert tr[0] == math.sqrt(kat2_rr0(*dims, s7=s7))  # KAT-2
    assert nr / tr[0] <= 1e-15
    assert (x - 1.0).abs().max().item() <= 1e-12
    if trace_iters:
        ref, pts = _oracle_trace(dims, s7, trace_iters)
        ref = np.asarray(ref)
        # every leading point above the 1e-20 cutoff (7-pt 256^3 passes it by k = 10)
        above = int(np.argmax(ref ** 2 < 1e-20 * ref[0] ** 2)) if np.any(ref ** 2 < 1e-20 * ref[0] ** 2) \
            else len(ref)
        assert above >= 10
        assert check_trace(tr, ref, RTRANS_RTOL_1GPU) == min(above, len(tr))
        used = "C restatement (oracle/hpccg_oracle.c)"
        if pts is not None:  # the reference build itself, where it is built (always here and on the GPU box)
            used = f"reference build oracle/_ref (OpenMP) at k = {sorted(pts)} + C restatement"
            for k, nr_ref in pts.items():
                rr, rr_ref = tr[k] ** 2, nr_ref ** 2
                if rr_ref >= 1e-20 * tr[0] ** 2:
                    assert abs(rr - rr_ref) <= RTRANS_RTOL_1GPU * rr_ref, (k, tr[k], nr_ref)
        record_property("oracle", used)
        print(f"test_full_size{dims}: oracle = {used}")


@pytest.mark.parametrize("dims,s7", [((1, 1, 1), False), ((2, 1, 1), False), ((3, 2, 1), False),
                                     ((1, 1, 700), False), ((31, 1, 1), False), ((1, 1, 1), True),
                                     ((2, 1, 1), True), ((3, 2, 1), True), ((1, 1, 700), True),
                                     ((31, 1, 1), True)])
def test_tiny_and_thin_grids(hp, gpu, dims, s7):
    """Degenerate grids (one row; lines; a slice-straddling 1x1x700 column),
    from the host and the device generator, against the oracle.

    When rtrans reaches exactly 0 the reference does one more iteration
    (HPCCG.cpp:358: the loop test is normr > tolerance, checked before the
    step) with p = 0, so alpha = 0/0 and x = x + NaN*0 (HPCCG.cpp:380-386):
    the reference returns NaN in x there, and so must we."""
    ref = oracle.hpccg(oracle.generate(*dims, use_7pt=s7), max_iter=50)
    prob = hp.generate_matrix(*dims, use_7pt=s7)
    for M in (hp.Matrix.from_hpc(prob), hp.Matrix.generate(*dims, use_7pt=s7)):
        x = prob.x  # a fresh copy of x0 each time
        _, it, nr, _ = hp.HPCCG(M, prob.b, x, max_iter=50)
        tr = M.last_trace()
        assert tr[0] == ref["trace"][0]
        check_final(it, nr, tr, ref["niters"], ref["normr"], ref["trace"], 50)
        if dims[0] * dims[1] * dims[2] <= 2:
            # exact arithmetic: r = 0 after one step, then the 0/0 step
            assert it == ref["niters"] and nr == 0.0
            assert np.isnan(x).all() and np.isnan(ref["x"]).all()
        elif not np.isnan(x).all():
            # 3x2x1: whether rtrans and p.Ap both underflow to 0 (-> NaN) in
            # the noise regime depends on the summation order
            assert np.max(np.abs(x - prob.xexact)) <= 1e-12


def _banded(n, vals_of, diag_first=True):
    """Symmetric 5-band matrix with the given off-diagonal value per (i, j)."""
    rp = [0]
    cols, vals = [], []
    for i in range(n):
        row = [(i, 0.0)]
        for j in (i - 7, i - 1, i + 1, i + 7):
            if 0 <= j < n:
                row.append((j, vals_of(min(i, j), max(i, j))))
        row[0] = (i, 4.5 + 2.0 * sum(abs(v) for _, v in row[1:]))  # well conditioned
        if not diag_first:
            row.sort()
        cols += [c for c, _ in row]
        vals += [v for _, v in row]
        rp.append(len(cols))
    return np.array(rp, np.int64), np.array(cols, np.int32), np.array(vals, np.float64)


def _random_patterns(n, seed, noffs=10, diag_first=True):
    """Symmetric matrix whose rows each keep a random subset of `noffs`
    offsets: few distinct offsets per slice, many holes."""
    rng = np.random.default_rng(seed)
    offs = [1, 2, 3, 5, 8, 13, 21, 34, 55, 89][:noffs]
    nb = [set() for _ in range(n)]
    for i in range(n):
        for o in offs:
            if rng.random() < 0.5 and i + o < n:
                nb[i].add(i + o)
                nb[i + o].add(i)
    rp = [0]
    cols, vals = [], []
    for i in range(n):
        row = [i] + sorted(nb[i]) if diag_first else sorted(nb[i] | {i})
        cols += row
        vals += [2.0 + len(row) if c == i else -1.0 for c in row]
        rp.append(len(cols))
    return np.array(rp, np.int64), np.array(cols, np.int32), np.array(vals, np.float64)


def test_sell_a_holes_and_refusal(hp, gpu, keep_sell):
    """SELL-512-A stores, per slice, one slot per distinct (column - row)
    offset in ascending order, 0.0 where a row has no entry. Rows with random
    offset subsets (many holes, x read past both ends of the vector for the
    first and last slices, a ragged last slice) give the SELL-512 bits on
    every kernel, fused or not; a matrix whose rows are not in ascending
    column order (diagonal first) gets no A image, since its sums would round
    in another order."""
    n = 2600  # 5 full slices + a ragged one
    rp, cols, vals = _random_patterns(n, 5, noffs=10, diag_first=False)
    M = hp.Matrix.from_csr(rp, cols, vals)
    assert M.get_option("has_a") == 1
    b = 1.0 + (np.arange(n) % 3)
    out = {}
    for kernel, fuse in itertools.product((SELL, DIRECT, PAIRS), (0, -1)):
        M.set_option("spmv_kernel", kernel)
        M.set_option("fuse_p", fuse)
        out[(kernel, fuse)] = solve_bits(hp, M, b, 70)
    assert all(o == out[(SELL, 0)] for o in out.values())
    A = oracle.CSR(rp, cols, vals, np.zeros(n), b, np.zeros(n))
    ref = oracle.hpccg(A, max_iter=70)
    assert check_trace(np.frombuffer(out[(SELL, 0)][2]), ref["trace"], RTRANS_RTOL_1GPU) >= 5
    # rows diagonal first: not ascending -> SELL-512 only
    rp, cols, vals = _banded(1500, lambda i, j: -1.0, diag_first=True)
    M = hp.Matrix.from_csr(rp, cols, vals)
    assert M.get_option("has_a") == 0 and M.get_option("spmv_kernel") == SELL
    with pytest.raises(hp.HPCCGError, match="not built"):
        M.set_option("spmv_kernel", PAIRS)
    # the same band sorted: an A image of width 5
    rp, cols, vals = _banded(1500, lambda i, j: -1.0 - ((i + j) % 5) * 0.25, diag_first=False)
    M = hp.Matrix.from_csr(rp, cols, vals)
    assert M.get_option("has_a") == 1 and M.get_option("a_width") == 5
    b = 1.0 + (np.arange(1500) % 7)
    A = oracle.CSR(rp, cols, vals, np.zeros(1500), b, np.zeros(1500))
    ref = oracle.hpccg(A, max_iter=40)
    got = solve_bits(hp, M, b, 40)
    assert check_trace(np.frombuffer(got[2]), ref["trace"], RTRANS_RTOL_1GPU) >= 5


def test_sell_a_offset_limit(hp, gpu):
    """A slice with more than 32 distinct offsets gets no SELL-512-A image; 32
    still fit (the limit is per slice, not per matrix)."""
    for noffs, fits in ((16, True), (40, False)):
        n = 2048
        offs = [3 * k + 1 for k in range(noffs // 2)]
        nb = [set() for _ in range(n)]
        for i in range(n):
            for o in offs:
                if i + o < n:
                    nb[i].add(i + o)
                    nb[i + o].add(i)
        rp, cols, vals = [0], [], []
        for i in range(n):
            row = sorted(nb[i] | {i})
            cols += row
            vals += [1.0 + len(row) if c == i else -1.0 for c in row]
            rp.append(len(cols))
        rp, cols, vals = np.array(rp, np.int64), np.array(cols, np.int32), np.array(vals, np.float64)
        M = hp.Matrix.from_csr(rp, cols, vals)
        assert M.get_option("has_a") == int(fits), noffs
        b = 1.0 + (np.arange(n) % 5)
        A = oracle.CSR(rp, cols, vals, np.zeros(n), b, np.zeros(n))
        ref = oracle.hpccg(A, max_iter=30)
        got = solve_bits(hp, M, b, 30)
        assert check_trace(np.frombuffer(got[2]), ref["trace"], RTRANS_RTOL_1GPU) >= 5
