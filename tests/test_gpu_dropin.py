"""The drop-in driver hpccg_hip_HPCCG (HPCCG.hpp:61-63 signature, C linkage):
the device matrix is cached per caller HPC_Sparse_Matrix, keyed by its
address AND a fingerprint of its contents, so a matrix edited in place (or
destroyed and re-created at the same address) is converted again; a matrix
that has been through the reference's make_local_matrix (local column
indices, local_ncol > local_nrow: make_local_matrix.cpp:595) is refused."""
import numpy as np
import pytest

import oracle
from conftest import RTRANS_RTOL_1GPU

pytestmark = pytest.mark.gpu


def test_dropin_cache_follows_the_contents(hp, gpu):
    prob = hp.generate_matrix(12, 10, 9)
    L = hp.lib()
    x = prob.x
    _, it, nr, _ = hp.dropin_HPCCG(prob, x, max_iter=200)
    assert L.hpccg_hip_dropin_cached(prob.A) == 1
    assert np.max(np.abs(x - 1.0)) <= 1e-12
    # same contents: the cached image, the same bits
    x2 = prob.x
    _, it2, nr2, _ = hp.dropin_HPCCG(prob, x2, max_iter=200)
    assert (it2, nr2) == (it, nr) and np.array_equal(x, x2)
    # edit the values in place (A -> 2A, same address): the solution of
    # 2A x = b is x = 1/2, a stale image would still give 1
    A = prob.A.contents
    nnz = int(sum(A.nnz_in_row[i] for i in range(A.local_nrow)))
    vals = np.ctypeslib.as_array(A.list_of_vals, (nnz,))
    vals *= 2.0
    x3 = prob.x
    hp.dropin_HPCCG(prob, x3, max_iter=200)
    assert np.max(np.abs(x3 - 0.5)) <= 1e-12
    # and the residual trajectory is the oracle's on the edited matrix
    rp, cols, vv = prob.to_csr()
    ref = oracle.hpccg(oracle.CSR(rp, cols, vv, np.zeros(len(x3)), prob.b, np.full(len(x3), 0.5)), max_iter=20)
    x4 = prob.x
    _, it4, nr4, _ = hp.dropin_HPCCG(prob, x4, max_iter=20)
    assert it4 == ref["niters"] and abs(nr4 ** 2 - ref["normr"] ** 2) <= RTRANS_RTOL_1GPU * ref["normr"] ** 2
    vals /= 2.0
    assert L.hpccg_hip_dropin_release(prob.A) == 1
    assert L.hpccg_hip_dropin_cached(prob.A) == 0
    assert L.hpccg_hip_dropin_release(prob.A) == 0


def test_dropin_refuses_a_localised_matrix(hp, gpu):
    prob = hp.generate_matrix(6, 6, 6)
    A = prob.A.contents
    A.local_ncol = A.local_nrow + 36  # as make_local_matrix.cpp:595 leaves it
    x = prob.x
    with pytest.raises(hp.HPCCGError, match="make_local_matrix"):
        hp.dropin_HPCCG(prob, x, max_iter=10)
    with pytest.raises(hp.HPCCGError, match="make_local_matrix"):
        hp.Matrix.from_hpc(prob)
    assert hp.lib().hpccg_hip_dropin_cached(prob.A) == 0
    A.local_ncol = A.local_nrow
    _, it, _, _ = hp.dropin_HPCCG(prob, x, max_iter=10)
    assert it == 9
    hp.lib().hpccg_hip_dropin_release(prob.A)


def test_dropin_new_matrix_same_address(hp, gpu):
    """Destroy and re-create: whatever address the new matrix gets, its
    solve is its own (the fingerprint differs: other sizes and values)."""
    for dims in ((8, 8, 8), (9, 7, 5), (8, 8, 8)):
        prob = hp.generate_matrix(*dims)
        x = prob.x
        _, it, nr, _ = hp.dropin_HPCCG(prob, x, max_iter=80)
        ref = oracle.hpccg(oracle.generate(*dims), max_iter=80)
        assert it == ref["niters"]
        assert abs(nr ** 2 - ref["normr"] ** 2) <= RTRANS_RTOL_1GPU * ref["normr"] ** 2 or ref["normr"] < 1e-12
        assert np.max(np.abs(x - 1.0)) <= 1e-12
        A = prob.A
        prob.close()  # hpccg_free_problem -> destroyMatrix -> hpccg_hip_dropin_release
        assert hp.lib().hpccg_hip_dropin_cached(A) == 0  # hpccg_free_problem -> destroyMatrix -> hpccg_hip_dropin_release


def test_dropin_prints_one_solve(hp, gpu, capfd):
    """A repeated call solves on the cached image while host threads
    fingerprint A (the fingerprint hidden under the solve); x and the
    reference's residual lines come out only once the fingerprint matched. An
    in-place edit found that way re-solves on a fresh image: the caller still
    sees ONE set of residual lines (HPCCG.cpp:356, 372-373), the edited
    matrix's."""
    prob = hp.generate_matrix(10, 9, 8)
    x = prob.x
    hp.dropin_HPCCG(prob, x, max_iter=50)  # builds and caches the image
    capfd.readouterr()
    x2 = prob.x
    _, it, nr, _ = hp.dropin_HPCCG(prob, x2, max_iter=50)  # cached: the speculative path
    out = capfd.readouterr().out
    assert out.count("Initial Residual") == 1 and out.count("Iteration = 49 ") == 1
    assert np.array_equal(x, x2)
    A = prob.A.contents
    nnz = int(sum(A.nnz_in_row[i] for i in range(A.local_nrow)))
    vals = np.ctypeslib.as_array(A.list_of_vals, (nnz,))
    vals *= 4.0
    x3 = prob.x
    _, it3, nr3, _ = hp.dropin_HPCCG(prob, x3, max_iter=50)
    out = capfd.readouterr().out
    assert out.count("Initial Residual") == 1, out
    assert np.max(np.abs(x3 - 0.25)) <= 1e-12  # the edited matrix's solution, not the stale image's
    vals /= 4.0
    hp.lib().hpccg_hip_dropin_release(prob.A)
