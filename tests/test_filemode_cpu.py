"""Mode 2 on the CPU: read_HPC_row (read_HPC_row.cpp:217-373) restated by
hpccg_read_HPC_row, and the oracle pinned on the file-mode golden solve.

The system comes from tests/golden/filemode.py (no RNG). Its golden trace is
the reference HPCCG() started from the file's initial guess, and
ref_cli_file_general_600.txt is the reference CLI (its own read_HPC_row.cpp)
run on the same file (tests/golden/make_golden.py)."""
import os
import sys

import numpy as np
import pytest

import oracle
from conftest import ROOT, check_final, check_trace, solve_case, unhex

sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import filemode  # noqa: E402


@pytest.fixture(scope="module")
def system_file(tmp_path_factory):
    rp, cl, vl, x0, b, xe = filemode.general_system(600)
    path = str(tmp_path_factory.mktemp("mode2") / "general_600.dat")
    filemode.write(path, rp, cl, vl, x0, b, xe)
    return path, (rp, cl, vl, x0, b, xe)


def block_partition(n, size, rank):
    """read_HPC_row.cpp:255-266."""
    chunk, rem = divmod(n, size)
    mp = chunk + (1 if rank < rem else 0)
    off = rank * (chunk + 1) - max(0, rank - rem)
    return off, mp


@pytest.mark.parametrize("size", [1, 2, 3, 7])
def test_reader_blocks_and_entries(hp, system_file, size):
    path, (rp, cl, vl, x0, b, xe) = system_file
    covered = 0
    for r in range(size):
        p = hp.read_HPC_row(path, r, size)
        off, mp = block_partition(600, size, r)
        assert (p.start_row, p.nrow, p.total_nrow, p.total_nnz) == (off, mp, 600, int(rp[-1]))
        rpl, cll, vll = p.to_csr()
        assert np.array_equal(rpl, rp[off:off + mp + 1] - rp[off])
        assert np.array_equal(cll, cl[rp[off]:rp[off + mp]])  # global columns, file order
        assert np.array_equal(vll, vl[rp[off]:rp[off + mp]])
        assert np.array_equal(p.x, x0[off:off + mp]) and np.array_equal(p.b, b[off:off + mp])
        assert np.array_equal(p.xexact, xe[off:off + mp])
        covered += mp
    assert covered == 600


def test_reader_errors(hp, tmp_path):
    with pytest.raises(hp.HPCCGError, match="Cannot open file"):
        hp.read_HPC_row(str(tmp_path / "missing.dat"))
    bad = tmp_path / "bad.dat"
    bad.write_text("3 5\n2\n2\n1\n2 4.0 0 -1.0 1\n")  # truncated
    with pytest.raises(hp.HPCCGError, match="read_HPC_row"):
        hp.read_HPC_row(str(bad))
    bad.write_text("2 2\n1\n1\n1 2.0 0\n1 2.0 7\n0 1 1\n0 1 1\n")  # column out of range
    with pytest.raises(hp.HPCCGError, match="bad entry"):
        hp.read_HPC_row(str(bad))


def test_oracle_file_mode_bitwise_reference(golden, system_file):
    """The oracle from the file's initial guess reproduces the reference trace
    bit for bit (serial order)."""
    _, (rp, cl, vl, x0, b, xe) = system_file
    c = solve_case(golden, "file_general_600")
    A = oracle.CSR(rp, cl, vl, x0, b, xe)
    ref_tr = [unhex(t) for t in c["trace_normr"]]
    for mi in (150, 500):
        r = oracle.hpccg(A, max_iter=mi)
        run = c["runs"][str(mi)]
        assert r["niters"] == run["niters"] and r["normr"] == unhex(run["normr"])
    r = oracle.hpccg(A, max_iter=len(ref_tr))
    assert [float(v) for v in r["trace"][:len(ref_tr)]] == ref_tr
    assert np.max(np.abs(r["x"] - xe)) <= 1e-12
