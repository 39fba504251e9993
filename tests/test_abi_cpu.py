"""CPU-only checks of the C-ABI library: it loads, exports every declared
symbol, and its host-side pieces (generator, SELL-512 builder, halo plan) are
right. No compute call touches a GPU here."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import oracle
from conftest import ROOT


def test_library_exports_every_declared_symbol(hp):
    L = hp.lib()
    declared = hp.exported_symbols()
    assert len(declared) >= 29
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    assert L.hpccg_hip_abi_version() == 2
    # and through the dynamic symbol table
    out = subprocess.run(["nm", "-D", "--defined-only", hp.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    for s in declared:
        assert f" T {s}" in out, s
    # C++ drop-in with the reference signature (HPCCG.hpp:61-63)
    assert "_Z5HPCCGP24HPC_Sparse_Matrix_STRUCTPdS1_idRiRdS1_" in out


def test_cli_built_and_usage(hp):
    assert os.path.exists(hp.CLI_PATH)
    r = subprocess.run([hp.CLI_PATH], capture_output=True, text=True)
    assert r.returncode == 1
    assert "Mode 1: " in r.stderr and "nx ny nz" in r.stderr


@pytest.mark.parametrize("dims,rank,size,s7", [((4, 3, 2), 0, 1, False), ((13, 7, 5), 0, 1, False),
                                               ((6, 5, 4), 1, 3, False), ((6, 5, 4), 2, 3, True),
                                               ((9, 8, 7), 0, 1, True), ((1, 1, 1), 0, 1, False)])
def test_host_generator_matches_oracle(hp, dims, rank, size, s7):
    prob = hp.generate_matrix(*dims, rank=rank, size=size, use_7pt=s7)
    rp, cols, vals = prob.to_csr()
    A = oracle.generate(*dims, rank=rank, size=size, use_7pt=s7)
    assert np.array_equal(rp, A.row_ptr)
    assert np.array_equal(cols, A.cols)
    assert np.array_equal(vals, A.vals)
    assert np.array_equal(prob.b, A.b)
    assert np.array_equal(prob.x, A.x) and np.array_equal(prob.xexact, A.xexact)
    S = prob.A.contents
    n = dims[0] * dims[1] * dims[2]
    assert (S.start_row, S.stop_row, S.total_nrow) == (n * rank, n * rank + n - 1, n * size)
    assert S.total_nnz == 27 * n * size  # generate_matrix.cpp:226 approximation kept
    # ptr_to_diags points at the 27.0 entry
    for i in range(min(n, 50)):
        assert S.ptr_to_diags[i][0] == 27.0


def test_host_generator_matches_reference_csr(hp, golden):
    g = golden["csr_4x3x2"]
    rp, cols, vals = hp.generate_matrix(4, 3, 2).to_csr()
    assert rp.tolist() == g["row_ptr"] and cols.tolist() == g["cols"] and vals.tolist() == g["vals"]


def _sell_reference(row_ptr, cols, vals, col_base, uniform):
    """Independent numpy statement of the SELL-512 image."""
    n = len(row_ptr) - 1
    ns = (n + 511) // 512
    lens = np.diff(row_ptr)
    w = np.array([lens[s * 512:(s + 1) * 512].max() if n else 0 for s in range(ns)], np.int64)
    if uniform:
        w[:] = w.max() if ns else 0
    base = np.concatenate([[0], np.cumsum(w)])
    sc = np.full(int(base[-1]) * 512, -1, np.int32)
    sv = np.zeros(int(base[-1]) * 512, np.float64)
    for i in range(n):
        s, lane = divmod(i, 512)
        for j in range(lens[i]):
            e = (base[s] + j) * 512 + lane
            sc[e] = cols[row_ptr[i] + j] - col_base
            sv[e] = vals[row_ptr[i] + j]
    return base.astype(np.uint32), sc, sv


@pytest.mark.parametrize("dims,s7", [((20, 20, 20), False), ((13, 7, 5), False), ((9, 8, 7), True)])
def test_sell_image(hp, dims, s7):
    A = oracle.generate(*dims, use_7pt=s7)
    sb, sc, sv = hp.sell_build(A.row_ptr, A.cols, A.vals)
    slots_var = sum(int(x) for x in np.diff(_sell_reference(A.row_ptr, A.cols, A.vals, 0, False)[0]))
    uniform = int(sb[-1]) * 512 == len(sc) and len(set(np.diff(sb))) <= 1
    rb, rc, rv = _sell_reference(A.row_ptr, A.cols, A.vals, 0, uniform)
    assert np.array_equal(sb, rb)
    assert np.array_equal(sc, rc) and np.array_equal(sv, rv)
    # SpMV from the image == oracle SpMV bitwise (same per-row order; padding adds +0)
    x = (np.arange(A.nrow) % 11) / 7.0 - 0.5
    n = A.nrow
    y = np.zeros(((n + 511) // 512) * 512)
    for s in range(len(sb) - 1):
        for j in range(int(sb[s + 1] - sb[s])):
            e0 = (int(sb[s]) + j) * 512
            c = sc[e0:e0 + 512]
            v = sv[e0:e0 + 512]
            xv = np.where(c >= 0, x[np.maximum(c, 0)], 0.0)
            y[s * 512:(s + 1) * 512] = y[s * 512:(s + 1) * 512] + v * xv
    assert np.array_equal(y[:n], oracle.sparsemv(A, x))
    assert slots_var <= int(sb[-1])


def test_halo_plan_for_slabs(hp):
    nx, ny, nz, P = 6, 5, 4, 4
    for r in range(P):
        A = oracle.generate(nx, ny, nz, rank=r, size=P)
        plan = hp.halo_plan(A.row_ptr, A.cols, A.start_row, A.total_nrow)
        assert plan["ghost_lo"] == (nx * ny if r > 0 else 0)
        assert plan["ghost_hi"] == (nx * ny if r < P - 1 else 0)


def test_device_calls_fail_loudly_without_gpu(hp):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(hp.HPCCGError):
        hp.Matrix.generate(8, 8, 8)
