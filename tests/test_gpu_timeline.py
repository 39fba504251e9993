"""The block-timeline diagnostic of the ring pair kernel (option dbg_timeline,
hpccg_hip_diag_timeline): it changes no value, records one row per slice
pair of the last iteration's launch, and its stamps are ordered. tools/
timeline.py turns it into the phase breakdown DESIGN.md section 4 cites."""
import numpy as np
import pytest

from test_gpu_parity import PAIRS, solve_bits

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dims,iters", [((40, 40, 40), 30), ((24, 20, 18), 7)])
def test_timeline_rows_and_bits(hp, gpu, dims, iters):
    prob = hp.generate_matrix(*dims)
    M = hp.Matrix.from_hpc(prob)
    M.set_option("spmv_kernel", PAIRS)
    assert M.get_option("a2_ring") == 3 and M.get_option("a_width") == 27
    base = solve_bits(hp, M, prob.b, iters)
    for graph in (1, 0):
        M.set_option("use_graph", graph)
        M.set_option("dbg_timeline", 1)
        assert M.get_option("dbg_timeline") == 1
        assert solve_bits(hp, M, prob.b, iters) == base  # diagnostics change no value
        tl = M.diag_timeline()
        M.set_option("dbg_timeline", 0)
        nslices = (dims[0] * dims[1] * dims[2] + 511) // 512
        units = (nslices + 1) // 2
        assert tl.shape[0] >= units
        rows = tl[:units]
        t = rows[:, 1:6].astype(np.int64)
        assert np.all(t > 0), "every pair recorded"
        assert np.all(np.diff(t, axis=1) >= 0), "entry <= state <= staged <= slots <= end"
        # the last launch that ran an iteration: k = iters - 1 (every pair of it)
        assert set(rows[:, 7].tolist()) == {iters - 1}
        # launch-wide span of one SpMV: well under a second of 100 MHz ticks
        assert 0 < t[:, 4].max() - t[:, 0].min() < 100_000_000
    with pytest.raises(hp.HPCCGError):
        M.diag_timeline()  # off again
    M.close()
