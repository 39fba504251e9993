import base64
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)


def unb64(s: str) -> np.ndarray:
    return np.frombuffer(base64.b64decode(s), dtype=np.float64).copy()


def unhex(s: str) -> float:
    return float.fromhex(s)


def solve_case(golden, name):
    for c in golden["solves"]:
        if c["name"] == name:
            return c
    raise KeyError(name)


# Stated fp64 parity tolerance ("Stated parity tolerance"):
#   every k with trace_ref[k]^2 >= 1e-20 * trace_ref[0]^2 must satisfy
#   |rtrans_gpu - rtrans_ref| <= RTRANS_RTOL * rtrans_ref  (rtrans = normr^2).
RTRANS_RTOL_1GPU = 1e-8
RTRANS_RTOL_MULTI = 1e-7
RTRANS_CUTOFF = 1e-20


CONVERGED_REL = 1e-15
# SURVEY 8c(4) asks |log10(normr_gpu / normr_ref)| <= 1 for the final residual.
# Stated deviation: that bar is applied only above the noise floor
# (normr_ref / normr0 > 1e-15), where check_final requires more (equal niters
# and 1e-4 relative). Below it the recurrence is rounding noise and the ratio
# is not a property of the implementation: the reference's own OpenMP build
# against its serial build gives ratios up to 10^1.14 (21 runs per case, see
# check_final), and the 8-rank summation order of 16x16x128 gives 10^2.13
# (1.76e-112 vs 2.35e-110, both ~1e-114 of normr0; GPU run of this round).
# There both runs must be in the noise regime instead.


def first_converged(tr):
    """First k with normr_k / normr_0 <= 1e-15 (the start of rounding noise)."""
    tr = np.asarray(tr, np.float64)
    hit = np.nonzero(tr <= CONVERGED_REL * tr[0])[0]
    return int(hit[0]) if len(hit) else None


def check_final(niters, normr, tr_test, ref_niters, ref_normr, ref_trace, max_iter):
    """Termination parity (stated tolerance).

    Before convergence the trajectory is checked by check_trace. After
    normr/normr0 <= 1e-15 the recurrence is rounding noise, and the reference
    itself is not reproducible there: its own OpenMP build (serial order vs
    2..8 threads, 21 runs each, measured with oracle/ in this repo) exits on
    rtrans underflow at niters 259..276 where serial gives 274 (10^3),
    268..279 vs 272 (13x7x5), 491..499 vs 499 (20^3), 319..499 vs 325
    (8x8x16), with final-residual ratios up to 10^1.14. So:
      * equal niters when both runs go the full max_iter-1 iterations;
      * otherwise (an underflow exit on either side) both runs must end in
        the noise regime;
      * both final residuals <= 1e-15 * normr0 (0 = underflow) whenever the
        reference's is;
      * the first converged iteration agrees within +-2.
    This replaces SURVEY 8c(4)'s |log10(normr_gpu/normr_ref)| <= 1 in the
    noise regime (stated deviation, see the comment above CONVERGED_REL's
    use); above it the check is stricter than 8c(4).
    """
    full = max_iter - 1
    r0 = tr_test[0]
    if ref_niters == full and niters == full:
        pass
    else:
        assert normr <= CONVERGED_REL * r0, (niters, normr)
        assert ref_normr <= CONVERGED_REL * r0, (ref_niters, ref_normr)
    if ref_normr <= CONVERGED_REL * r0:
        assert normr <= CONVERGED_REL * r0, (normr, r0)
    else:
        assert niters == ref_niters
        assert abs(normr - ref_normr) <= 1e-4 * ref_normr, (normr, ref_normr)
    kt, kr = first_converged(tr_test), first_converged(ref_trace)
    if kr is not None and kt is not None:
        assert abs(kt - kr) <= 2, (kt, kr)


def check_trace(tr_test, tr_ref, rtol):
    """Phase-aware trace comparison on rtrans = normr^2. Returns #points checked."""
    tr_test = np.asarray(tr_test, np.float64)
    tr_ref = np.asarray(tr_ref, np.float64)
    r0 = tr_ref[0] ** 2
    m = min(len(tr_test), len(tr_ref))
    checked = 0
    for k in range(m):
        rr = tr_ref[k] ** 2
        if rr < RTRANS_CUTOFF * r0:
            break
        rt = tr_test[k] ** 2
        assert abs(rt - rr) <= rtol * rr, (k, rt, rr, abs(rt - rr) / rr)
        checked += 1
    return checked


def kat2_rr0(nx, ny, nz, s7=False):
    """KAT-2: rtrans_0 = sum over rows of b_i^2 = (28 - nnz_i)^2
    (generate_matrix.cpp:259-286), exact in integers. 27-pt: nnz_i is the
    product of the per-axis counts (2 at a face, 3 inside, 1 on a 1-wide
    axis); 7-pt: 1 + the per-axis neighbour counts."""
    def axis(n):
        c = np.full(n, 3, np.int64)
        c[0] -= 1
        c[-1] -= 1
        if n == 1:
            c[0] = 1
        return np.unique(c, return_counts=True)
    tot = 0
    for cx, nx_ in zip(*axis(nx)):
        for cy, ny_ in zip(*axis(ny)):
            for cz, nz_ in zip(*axis(nz)):
                nnz = (cx - 1) + (cy - 1) + (cz - 1) + 1 if s7 else cx * cy * cz
                tot += int(nx_) * int(ny_) * int(nz_) * (28 - int(nnz)) ** 2
    return tot


def load_pkg():
    """Import hpccg-sycl_amd/ (hyphenated dir) as module hpccg_sycl_amd."""
    import importlib.util
    name = "hpccg_sycl_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(
        name, os.path.join(ROOT, "hpccg-sycl_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def hp():
    return load_pkg()


@pytest.fixture(scope="session")
def gpu(hp):
    """GPU tests: the HIP library must load and see a device -- no fallback."""
    import torch
    assert torch.cuda.is_available(), "gpu test without a visible HIP device"
    hp.lib()
    assert hp.device_count() >= 1
    hp.set_device(0)
    return torch.device("cuda:0")
