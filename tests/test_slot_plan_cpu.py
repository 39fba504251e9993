"""Host checks of the folded dot completion's waiter choice (no GPU).

The slot completion (hpccg_kernels.hip, complete_dot_lanes) lets exactly one
block of each group of 64 slices wait for the group's partials, and one of
those waiters wait for every group sum. The wait always ends only if every
block it waits for was dispatched before it, i.e. has a smaller block index
(workgroups are dispatched in index order on every XCD). These tests run the
library's own plan (the functions the kernels call, compiled for the host)
over many launch shapes and check that property by brute force against the
block mapping xcd_slice / xcd_slice_rev: unit u of the x-th eighth
(per = grid / 8 units each) at position i runs in block 8 i + x, or
8 (per - 1 - i) + x reversed."""
import itertools

import pytest


def block_of(u, per, rev):
    x, i = divmod(u, per)
    return 8 * ((per - 1 - i) if rev else i) + x


def grid_of(units):
    return max(8, (units + 7) // 8 * 8)


SHAPES = sorted({1, 2, 7, 8, 9, 63, 64, 65, 100, 127, 128, 129, 977, 1000, 1954, 1800, 3907, 7813, 15625})


@pytest.mark.parametrize("units", SHAPES)
def test_waiters_wait_only_for_earlier_blocks(hp, units):
    for spu, rev in itertools.product((1, 2), (False, True)):
        if spu == 2 and rev:
            continue  # the pair kernel never walks backwards
        grid = grid_of(units)
        per = grid // 8
        last, top = hp.slot_plan(units, grid, spu, rev)
        upg = 64 // spu
        ng = (units * spu + 63) // 64
        assert len(last) == ng
        for g in range(ng):
            members = range(g * upg, min(units, (g + 1) * upg))
            bw = block_of(last[g], per, rev)
            assert last[g] in members
            assert all(block_of(u, per, rev) <= bw for u in members), (units, spu, rev, g)
        assert 0 <= top < ng
        bt = block_of(last[top], per, rev)
        assert all(block_of(last[g], per, rev) <= bt for g in range(ng)), (units, spu, rev)


def test_plan_rejects_bad_shapes(hp):
    with pytest.raises(hp.HPCCGError):
        hp.slot_plan(10, 12, 1)  # grid not a multiple of 8
    with pytest.raises(hp.HPCCGError):
        hp.slot_plan(100, 64, 1)  # fewer blocks than units
