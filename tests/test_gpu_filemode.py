"""Mode 2 and the gather halo plan on the GPU.

* one GPU: read_HPC_row -> HPC_Sparse_Matrix -> HPCCG from the file's initial
  guess, against the reference trace (golden file_general_600);
* P ranks (in-process group, the multi-rank kernels): the block partition of
  read_HPC_row.cpp:255-266 needs columns from non-adjacent ranks, so the
  library builds the gather plan (make_local_matrix.cpp:58-610: externals
  after the local rows, grouped by owner; exchange_externals.cpp:51-131 packs
  the requested rows) -- against the same serial reference trace (1e-7);
* the gather plan forced on a z-slab problem gives the slab plan's bits;
* the CLI in Mode 2 against the reference CLI's output on the same file."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import (ROOT, RTRANS_RTOL_1GPU, RTRANS_RTOL_MULTI, check_final, check_trace,
                      solve_case, unhex)

sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import filemode  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def system_file(tmp_path_factory):
    rp, cl, vl, x0, b, xe = filemode.general_system(600)
    path = str(tmp_path_factory.mktemp("mode2g") / "general_600.dat")
    filemode.write(path, rp, cl, vl, x0, b, xe)
    return path


def _ref(golden):
    c = solve_case(golden, "file_general_600")
    return c, [unhex(t) for t in c["trace_normr"]]


def test_file_mode_one_gpu(hp, gpu, golden, system_file):
    c, ref_tr = _ref(golden)
    p = hp.read_HPC_row(system_file)
    M = hp.Matrix.from_hpc(p)
    for mi in (150, 500):
        x = p.x  # the file's initial guess
        _, it, nr, _ = hp.HPCCG(M, p.b, x, max_iter=mi)
        tr = M.last_trace()
        assert tr[0] == ref_tr[0]
        assert check_trace(tr, ref_tr, RTRANS_RTOL_1GPU) >= 10
        run = c["runs"][str(mi)]
        check_final(it, nr, tr, run["niters"], unhex(run["normr"]), ref_tr, mi)
        assert np.max(np.abs(x - p.xexact)) <= 1e-12


def _group_solve(hp, gpu, probs, Ms, max_iter):
    import torch
    xs = [torch.from_numpy(p.x).to(gpu) for p in probs]
    bs = [torch.from_numpy(p.b).to(gpu) for p in probs]
    _, it, nr, times = hp.group_HPCCG(Ms, bs, xs, max_iter=max_iter)
    return it, nr, [x.cpu().numpy() for x in xs], times


@pytest.mark.parametrize("P", [2, 3, 4])
def test_file_mode_ranks_gather_plan(hp, gpu, golden, system_file, P):
    c, ref_tr = _ref(golden)
    probs = [hp.read_HPC_row(system_file, r, P) for r in range(P)]
    parts = [(*p.to_csr(), p.start_row) for p in probs]
    Ms = hp.group_from_csr(parts, 600)
    for M in Ms:
        # P >= 3: rank 0 needs rows of the last rank -> gather plan; P = 2: the
        # neighbour owns everything else, the slab plan serves (whole-block ghosts)
        assert M.get_option("halo_mode") == (2 if P >= 3 else 1)
        assert M.get_option("num_external") > 0
    it, nr, xs, times = _group_solve(hp, gpu, probs, Ms, 500)
    tr = Ms[0].last_trace()
    assert tr[0] == ref_tr[0]
    assert check_trace(tr, ref_tr, RTRANS_RTOL_MULTI) >= 10
    run = c["runs"]["500"]
    check_final(it, nr, tr, run["niters"], unhex(run["normr"]), ref_tr, 500)
    for p, x in zip(probs, xs):
        assert np.max(np.abs(x - p.xexact)) <= 1e-12
    assert times[5] > 0.0


def test_gather_plan_equals_slab_plan_bitwise(hp, gpu):
    """The same z-slab problem with the slab plan and with the gather plan
    forced: only the transport differs, every value is the same."""
    nx, ny, nz, P = 9, 8, 6, 3
    parts = []
    for r in range(P):
        prob = hp.generate_matrix(nx, ny, nz, rank=r, size=P)
        parts.append((*prob.to_csr(), r * nx * ny * nz, prob))
    out = []
    try:
        for mode in (1, 2):
            hp.set_halo_mode(mode)
            Ms = hp.group_from_csr([q[:4] for q in parts], P * nx * ny * nz)
            assert Ms[1].get_option("halo_mode") == mode
            for fuse in (0, 1):
                for M in Ms:
                    M.set_option("fuse_p", fuse)
                it, nr, xs, _ = _group_solve(hp, gpu, [q[4] for q in parts], Ms, 80)
                out.append((it, nr, Ms[0].last_trace().tobytes(), b"".join(x.tobytes() for x in xs)))
    finally:
        hp.set_halo_mode(0)
    assert all(o == out[0] for o in out)


def test_file_mode_cli_matches_reference(hp, gpu, tmp_path, system_file):
    exe = os.path.join(ROOT, "hpccg-sycl_amd", "bin", "test_HPCCG")
    r = subprocess.run([exe, system_file], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = r.stdout.splitlines()
    ref = open(os.path.join(ROOT, "tests", "golden", "ref_cli_file_general_600.txt")).read()
    ref = ref.replace("<DATA_FILE>", system_file).splitlines()
    assert out[0] == ref[0]  # "Reading matrix info from <file>..."
    assert out[1] == ref[1]  # initial residual, %g
    res_o = [l.split("Residual")[0] for l in out if l.startswith("Iteration =")]
    res_r = [l.split("Residual")[0] for l in ref if l.startswith("Iteration =")]
    m = min(len(res_o), len(res_r))  # the underflow exit is rounding noise
    assert res_o[:m] == res_r[:m] and m >= 5
    keys = lambda ls: [l.split(":")[0] for l in ls if ":" in l and not l.startswith(("Iteration", "Elapsed", "Reading", "Initial"))]
    ko, kr = keys(out), keys(ref)
    assert ko[:len(kr)] == kr  # same YAML keys in the same order; ours appends GPU Summary
    for k in ("  nx", "  ny", "  nz"):
        assert next(l for l in out if l.startswith(k + ":")) == k + ": 0"
    it = int(next(l for l in out if l.startswith("Number of iterations")).split(":")[1])
    fl = out.index("FLOPS Summary: ")
    assert out[fl + 4] == "  SPARSEMV: %g" % (it * 2.0 * 4200)  # file's total_nnz, main.cpp:222-226
    diff = float(next(l for l in out if "Difference between computed and exact" in l).split(":")[1])
    assert diff <= 1e-12


def test_file_mode_cli_missing_file(hp, gpu, tmp_path):
    exe = os.path.join(ROOT, "hpccg-sycl_amd", "bin", "test_HPCCG")
    r = subprocess.run([exe, str(tmp_path / "nope.dat")], cwd=tmp_path, capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 1
    assert "Error: Cannot open file" in r.stdout
