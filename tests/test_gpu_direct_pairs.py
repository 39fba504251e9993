"""The direct kernel over slice pairs (k_spmv_a2s, option direct_spu 2;
automatic where one block per slice needs between one and two rounds of
resident blocks, e.g. 100^3): each block runs two slices with k_spmv_a's
exact per-slice arithmetic, so every solve is bitwise the one-slice kernel's
-- fused update on and off, graph and eager, odd slice counts, and the prologue
(HPC_sparsemv.cpp:68-89, ddot.cpp:60-73)."""
import pytest

from test_gpu_parity import DIRECT, solve_bits

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dims", [(40, 36, 30), (32, 32, 31), (16, 16, 16)])
@pytest.mark.parametrize("opts", [{}, {"fuse_update": 0}, {"use_graph": 0}, {"x_defer": 1}])
def test_direct_pairs_bitwise(hp, gpu, dims, opts):
    prob = hp.generate_matrix(*dims)
    out = {}
    for spu in (1, 2):
        M = hp.Matrix.from_hpc(prob)
        M.set_option("spmv_kernel", DIRECT)
        M.set_option("direct_spu", spu)
        for k, v in opts.items():
            M.set_option(k, v)
        assert M.get_option("direct_spu") == spu
        out[spu] = solve_bits(hp, M, prob.b, 70)
        M.close()
    assert out[1] == out[2]


def test_direct_pairs_auto_at_100(hp, gpu):
    """100^3 (1954 slices) takes the pair form by default; 40x36x30 does not."""
    M = hp.Matrix.generate(100, 100, 100)
    assert M.get_option("spmv_kernel") == DIRECT and M.get_option("direct_spu") == 2
    M.close()
    M = hp.Matrix.generate(40, 36, 30)
    assert M.get_option("direct_spu") == 1
    M.close()
