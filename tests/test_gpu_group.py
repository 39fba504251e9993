"""Multi-rank kernels on the GPU: the in-process rank group.

RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), so a 1-GPU box
cannot run the RCCL job itself. hpccg_hip_group_* drives the same z-slab
ranks from one thread instead: every member is built and solved by the
multi-rank code path (ghost-localised columns, LDS windows over the ghost
planes, the all-reduced scalars in g, cg_run on all-reduced values, one
hipGraph for all members on one device), and only the transport differs (peer copies of the ghost planes, a rank-ordered sum for
the two scalars). The oracle is the serial reference run of the z-stacked
global problem (SURVEY 4 "Multi-GPU oracle"; golden cases *_xNranks,
generate_matrix.cpp:225-229), tolerance RTRANS_RTOL_MULTI."""
import itertools
import math

import numpy as np
import pytest

from conftest import RTRANS_RTOL_MULTI, check_final, check_trace, kat2_rr0, solve_case, unhex

pytestmark = pytest.mark.gpu


def _solve_group(hp, Ms, max_iter=500, tol=0.0, bs=None):
    import torch
    xs = [torch.zeros(M.info()["nrow"], dtype=torch.float64, device="cuda:0") for M in Ms]
    if bs is None:
        bs = [M.vectors()[0] for M in Ms]
    ierr, niters, normr, times = hp.group_HPCCG(Ms, bs, xs, max_iter=max_iter, tolerance=tol)
    return niters, normr, [x.cpu().numpy() for x in xs], times


@pytest.mark.parametrize("name", ["27pt_16x16x16_x8ranks", "27pt_8x8x8_x2ranks",
                                  "7pt_12x10x8_x2ranks"])
def test_group_matches_global_reference(hp, gpu, golden, name):
    c = solve_case(golden, name)
    P = c["ranks"]
    Ms = hp.group_generate(c["nx"], c["ny"], c["nz"], P, use_7pt=c["use_7pt"])
    nxy = c["nx"] * c["ny"]
    for r, M in enumerate(Ms):
        inf = M.info()
        assert inf["ghost_lo"] == (nxy if r > 0 else 0)
        assert inf["ghost_hi"] == (nxy if r < P - 1 else 0)
    niters, normr, xs, times = _solve_group(hp, Ms)
    ref_tr = [unhex(t) for t in c["trace_normr"]]
    rr = c["runs"]["500"]
    tr = Ms[0].last_trace()
    for M in Ms[1:]:
        assert np.array_equal(M.last_trace(), tr)  # one set of all-reduced scalars
    assert tr[0] == ref_tr[0]
    assert check_trace(tr, ref_tr, RTRANS_RTOL_MULTI) >= 5
    check_final(niters, normr, tr, rr["niters"], unhex(rr["normr"]), ref_tr, 500)
    assert max(np.max(np.abs(x - 1.0)) for x in xs) <= 1e-12
    assert times[5] > 0.0 and times[4] > 0.0  # halo and all-reduce classes were stamped


def test_group_kernel_variants_bitwise(hp, gpu):
    """Multi-rank SpMV kernels (SELL-512 gather, SELL-512-A direct, SELL-512-A
    pair windows whose windows include the ghost planes), the p update fused
    into the pair and direct kernels (r's halo lands in r's ghost planes), the
    dot completion modes, the deferred x update and graph replay give the same
    bits."""
    hp.set_keep_sell(True)
    try:
        Ms = hp.group_generate(24, 20, 9, 3)
    finally:
        hp.set_keep_sell(False)
    ref = None
    for kernel, fold, fuse, defer, graph in itertools.product((2, 1, 0), (0, 1), (0, -1), (0, 1, 2), (0, 1)):
        for M in Ms:
            M.set_option("spmv_kernel", kernel)
            M.set_option("fold", fold)
            M.set_option("fuse_p", fuse)
            M.set_option("x_defer", defer)
            M.set_option("use_graph", graph)
        # p = r + beta p inside the SpMV on multiple ranks: the pair kernel, and the
        # direct kernel with the halo received into r's ghost planes (z-slab plan)
        assert Ms[1].get_option("fuse_p") == (1 if (fuse and kernel in (1, 2)) else 0)
        niters, normr, xs, _ = _solve_group(hp, Ms, max_iter=90)
        if graph:
            assert Ms[0].get_option("graph_used") == 1
        got = (niters, normr, Ms[0].last_trace().tobytes(), b"".join(x.tobytes() for x in xs))
        if ref is None:
            ref = got
        if got != ref:  # (a plain assert would diff megabytes of bytes)
            pytest.fail(f"{(kernel, fold, fuse, defer, graph)}: niters {got[0]} vs {ref[0]}, normr {got[1]} "
                        f"vs {ref[1]}, trace equal {got[2] == ref[2]}")
    # the x ring length and graph chunk (a multiple of the ring with a halo)
    for ring, chunk, fold in ((5, 8, 1), (16, 3, 1), (-1, 8, 0), (32, 1, 0), (2, 13, 1)):
        for M in Ms:
            M.set_option("spmv_kernel", -1)
            M.set_option("fuse_p", -1)
            M.set_option("x_defer", 1 + ring % 2)  # batched / staggered
            M.set_option("x_ring", ring)
            M.set_option("graph_chunk", chunk)
            M.set_option("fold", fold)
        niters, normr, xs, _ = _solve_group(hp, Ms, max_iter=90)
        got = (niters, normr, Ms[0].last_trace().tobytes(), b"".join(x.tobytes() for x in xs))
        if got != ref:
            pytest.fail(f"{(ring, chunk, fold)}: niters {got[0]} vs {ref[0]}, normr {got[1]} vs {ref[1]}")
    assert Ms[0].get_option("lds_doubles") > 0


def test_group_8x200_weak_scaled(hp, gpu):
    """BASELINE configs[3] on the HIP path: 8 z-stacked ranks of local 200^3
    (global 200 x 200 x 1600, generate_matrix.cpp:225-229), every rank the
    multi-rank kernels (pair windows over the ghost planes, k_p_boundary, the
    halo in line, all-reduced scalars), all eight on this one GPU (about 4.2 GB each),
    graph-replayed. KAT-4 on the global nnz, KAT-2 (rtrans_0 exact), the full
    499 iterations, one trace on every rank, the final residual and x."""
    import torch
    P, nx = 8, 200
    Ms = hp.group_generate(nx, nx, nx, P)
    nnz = sum(M.info()["nnz"] for M in Ms)
    assert nnz == 1715783992  # (3*200-2)^2 * (3*1600-2)
    for r, M in enumerate(Ms):
        assert M.get_option("spmv_kernel") == 2
        assert M.get_option("device_bytes") <= 4.6e9
    niters, normr, xs, times = _solve_group(hp, Ms, max_iter=500)
    assert Ms[0].get_option("graph_used") == 1
    assert niters == 499
    tr = Ms[0].last_trace()
    for M in Ms[1:]:
        assert np.array_equal(M.last_trace(), tr)
    assert tr[0] == math.sqrt(kat2_rr0(nx, nx, P * nx))
    assert normr / tr[0] <= 1e-15
    assert max(np.max(np.abs(x - 1.0)) for x in xs) <= 1e-12
    assert times[4] > 0.0 and times[5] > 0.0
    del xs
    for M in Ms:
        M.close()
    torch.cuda.empty_cache()


def test_group_from_host_csr_equals_device_generator(hp, gpu):
    """Host generate_matrix per rank (global columns) -> group_from_csr: same
    SELL image, same solve bits as the device generator."""
    nx, ny, nz, P = 10, 9, 7, 3
    parts = []
    for r in range(P):
        prob = hp.generate_matrix(nx, ny, nz, rank=r, size=P)
        rp, cols, vals = prob.to_csr()
        parts.append((rp, cols, vals, r * nx * ny * nz))
    Mh = hp.group_from_csr(parts, P * nx * ny * nz)
    Md = hp.group_generate(nx, ny, nz, P)
    for a, b in zip(Mh, Md):
        assert a.info() == b.info()
    bs = [M.vectors()[0] for M in Md]  # device generator's b == generate_matrix's b
    r1 = _solve_group(hp, Mh, max_iter=100, bs=bs)
    r2 = _solve_group(hp, Md, max_iter=100)
    assert r1[0] == r2[0] and r1[1] == r2[1]
    assert Mh[0].last_trace().tobytes() == Md[0].last_trace().tobytes()
    assert all(np.array_equal(a, b) for a, b in zip(r1[2], r2[2]))


def test_group_of_one_equals_single_rank(hp, gpu):
    (Mg,) = hp.group_generate(12, 11, 10, 1)
    niters, normr, xs, _ = _solve_group(hp, [Mg], max_iter=120)
    M = hp.Matrix.generate(12, 11, 10)
    import torch
    b, _, _ = M.vectors()
    x = torch.zeros(12 * 11 * 10, dtype=torch.float64, device="cuda:0")
    _, it, nr, _ = hp.HPCCG(M, b, x, max_iter=120, device=True)
    assert (it, nr) == (niters, normr)
    assert M.last_trace().tobytes() == Mg.last_trace().tobytes()
    assert np.array_equal(x.cpu().numpy(), xs[0])


def test_group_errors(hp, gpu):
    Ms = hp.group_generate(6, 6, 4, 2)
    import torch
    b, _, _ = Ms[0].vectors()
    x = torch.zeros(144, dtype=torch.float64, device="cuda:0")
    with pytest.raises(hp.HPCCGError, match="group"):
        hp.HPCCG(Ms[0], b, x, max_iter=10, device=True)  # a member alone
    with pytest.raises(hp.HPCCGError):
        hp.group_HPCCG(Ms[::-1], [b, b], [x, x], max_iter=10)  # wrong rank order
    with pytest.raises(hp.HPCCGError):
        hp.group_generate(6, 6, 4, 17)  # more than 16 ranks


@pytest.mark.parametrize("nx,ny,nz,P,s7", [(33, 17, 9, 3, False), (7, 5, 1, 4, False), (1, 9, 6, 2, True),
                                           (19, 1, 3, 5, True), (40, 30, 2, 6, False)])
def test_group_odd_shapes_vs_oracle(hp, gpu, nx, ny, nz, P, s7):
    """Odd and degenerate slabs (one plane per rank: the ghosts are the whole
    neighbours; nx or ny = 1; partial last slices) against the serial oracle of
    the z-stacked global problem (SURVEY 4 multi-GPU oracle), 1e-7."""
    import oracle
    Ms = hp.group_generate(nx, ny, nz, P, use_7pt=s7)
    niters, normr, xs, _ = _solve_group(hp, Ms, max_iter=120)
    ref = oracle.hpccg(oracle.generate(nx, ny, nz * P, use_7pt=s7), max_iter=120)
    tr = Ms[0].last_trace()
    assert tr[0] == ref["trace"][0]
    assert check_trace(tr, ref["trace"], RTRANS_RTOL_MULTI) >= 3
    check_final(niters, normr, tr, ref["niters"], ref["normr"], ref["trace"], 120)
    x = np.concatenate(xs)
    assert np.max(np.abs(x - 1.0)) <= 1e-12 or ref["normr"] > 1e-15 * ref["trace"][0]
