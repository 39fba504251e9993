"""The CLI seam on the GPU: our test_HPCCG and the reference's own main.cpp
linked against libhpccg_hip.so (oracle/_ref/test_HPCCG_dropin) must print what
the reference CLI prints (tests/golden/ref_cli_*.txt): same lines, same YAML
keys, identical deterministic values (dimensions, iterations, FLOPS), the
initial residual bit-identical at %g, residual lines at the same iterations."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

DROPIN = os.path.join(ROOT, "oracle", "_ref", "test_HPCCG_dropin")


def keys(text):
    """YAML key paths (indent-aware), timing values dropped."""
    out = []
    for line in text.splitlines():
        m = re.match(r"^( *)([^:]+): ?(.*)$", line)
        if m and not line.startswith(("Initial Residual", "Iteration", "Elapsed")):
            out.append((len(m.group(1)), m.group(2)))
    return out


def values(text):
    d = {}
    path = []
    for line in text.splitlines():
        m = re.match(r"^( *)([^:]+): ?(.*)$", line)
        if not m or line.startswith(("Initial Residual", "Iteration", "Elapsed")):
            continue
        lvl = len(m.group(1)) // 2
        path = path[:lvl] + [m.group(2)]
        d["/".join(path)] = m.group(3)
    return d


def run_cli(exe, dims, tmp_path, env=None):
    e = dict(os.environ)
    e.update(env or {})
    r = subprocess.run([exe, *map(str, dims)], cwd=tmp_path, capture_output=True, text=True,
                       env=e, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout


def residual_lines(text):
    return [l for l in text.splitlines() if l.startswith(("Initial Residual", "Iteration ="))]


def compare_to_reference(out, ref, extra_ok=("GPU Summary",)):
    # residual lines: same iterations printed, initial residual identical
    lo, lr = residual_lines(out), residual_lines(ref)
    m = min(len(lo), len(lr))  # an underflow exit may end the listing earlier
    assert [l.split("Residual")[0] for l in lo[:m]] == [l.split("Residual")[0] for l in lr[:m]]
    assert m >= len(lr) - 1
    assert lo[0] == lr[0]
    assert any(l.startswith("Elapsed time: ") and l.endswith(" s") for l in out.splitlines())
    ko = [k for k in keys(out)]
    kr = keys(ref)
    # our extra block is appended at the end
    if ko != kr:
        cut = next(i for i, k in enumerate(ko) if k[1] in extra_ok)
        assert ko[:cut] == kr
    vo, vr = values(out), values(ref)
    fo, fr = float(vo["Final residual"]), float(vr["Final residual"])
    r0 = float(lo[0].split("=")[1])
    assert fo <= 1e-15 * r0 and fr <= 1e-15 * r0
    same = ["Dimensions/nx", "Dimensions/ny", "Dimensions/nz", "Mini-Application Name",
            "Mini-Application Version"]
    if fr > 0.0:  # no underflow exit: the iteration count and FLOPS are equal
        same += ["Number of iterations", "FLOPS Summary/Total   ", "FLOPS Summary/DDOT    ",
                 "FLOPS Summary/WAXPBY  ", "FLOPS Summary/SPARSEMV"]
    else:
        # rtrans underflow exit: iteration is rounding noise (the
        # reference's own OpenMP build exits at 259..276 for 10^3); FLOPS follow
        # main.cpp:224-226 from our own count
        it = int(vo["Number of iterations"])
        n = int(vo["Dimensions/nx"]) * int(vo["Dimensions/ny"]) * int(vo["Dimensions/nz"])
        assert 240 <= it <= 300
        assert vo["FLOPS Summary/DDOT    "] == "%g" % (it * 4.0 * n)
        assert vo["FLOPS Summary/SPARSEMV"] == "%g" % (it * 2.0 * 27 * n)
        assert fo == 0.0 or fo <= 1e-15 * r0
    for k in same:
        assert vo[k] == vr[k], k


@pytest.mark.parametrize("dims", [(20, 20, 20), (10, 10, 10)])
def test_our_cli_matches_reference_output(gpu, tmp_path, dims):
    out = run_cli(os.path.join(ROOT, "hpccg-sycl_amd", "bin", "test_HPCCG"), dims, tmp_path)
    ref = open(os.path.join(ROOT, "tests", "golden", "ref_cli_%dx%dx%d.txt" % dims)).read()
    compare_to_reference(out, ref)
    assert any(f.startswith("hpccg-1.0_") and f.endswith(".yaml") for f in os.listdir(tmp_path))
    v = values(out)
    assert float(v["GPU Summary/Difference between computed and exact"]) <= 1e-12


def test_our_cli_device_generator_and_max_iter_env(gpu, tmp_path):
    out = run_cli(os.path.join(ROOT, "hpccg-sycl_amd", "bin", "test_HPCCG"), (10, 10, 10), tmp_path,
                  env={"HPCCG_DEVICE_GENERATE": "1", "HPCCG_MAX_ITER": "150"})
    ref = open(os.path.join(ROOT, "tests", "golden", "out_10x10x10_150.txt")).read()
    lo = residual_lines(out)
    assert lo[0] == "Initial Residual = 258.24"
    assert lo[1] == "Iteration = 15   Residual = 2.15402e-06"  # out.txt:2, pre-convergence
    assert [l.split("Residual")[0] for l in lo] == [l.split("Residual")[0]
                                                      for l in residual_lines(ref)]
    assert values(out)["Number of iterations"] == "149"


@pytest.mark.skipif(not os.path.exists(DROPIN), reason="oracle/_ref/test_HPCCG_dropin not built")
def test_reference_main_linked_to_our_library(gpu, tmp_path):
    """the reference's own main.cpp, generate_matrix.cpp and
    YAML code, with HPCCG() resolved from libhpccg_hip.so, on the GPU."""
    out = run_cli(DROPIN, (20, 20, 20), tmp_path)
    ref = open(os.path.join(ROOT, "tests", "golden", "ref_cli_20x20x20.txt")).read()
    compare_to_reference(out, ref)
    assert keys(out) == keys(ref)  # the reference's own report code: exact key set


def test_cli_yaml_fractions_at_200(hp, gpu, tmp_path):
    """the CLI's GPU Summary reports the
    format-compulsory fraction of the 8 TB/s peak (<= 1) and SURVEY 8(d)'s
    credited bytes as bytes only (more than the format moves at 200^3:
    SELL-512-A stores no per-entry column), and the compulsory fraction is
    bench.py's roofline figure:
    the same bytes (bench.py adds the side blocks', which run after the p.Ap
    total, outside the CLI's class) over the launch time, within 5 % of the
    bench's frac measured the bench's way (hipEvents around the SpMV launch of
    an eager solve) when the CLI's definition is evaluated in this process;
    the CLI itself is another process, and the physical placement a process
    draws moves the 200^3 launch by up to ~7-14 % between processes on one box
    (DESIGN 4), so the direct cross-process comparison is held to 25 %."""
    out = run_cli(os.path.join(ROOT, "hpccg-sycl_amd", "bin", "test_HPCCG"), (200, 200, 200), tmp_path,
                  env={"HPCCG_DEVICE_GENERATE": "1", "HPCCG_MAX_ITER": "120"})
    v = values(out)
    comp = float(v["GPU Summary/SPARSEMV compulsory fraction of 8 TB/s HBM peak"])
    cred = float(v["GPU Summary/SPARSEMV credited bytes per call (SURVEY 12 nnz + 20 n)"])
    assert 0.3 < comp <= 1.0, comp
    assert not any("credited fraction" in k or "credited GB/s" in k for k in v)
    import torch
    M = hp.Matrix.generate(200, 200, 200)
    b, _, _ = M.vectors()
    n = 200 ** 3
    x = torch.zeros(n, dtype=torch.float64, device=gpu)
    hp.HPCCG(M, b, x, max_iter=40, device=True)  # warm
    x.zero_()
    _, it_g, _, t_g = hp.HPCCG(M, b, x, max_iter=120, device=True)  # graph replay, as the CLI runs
    M.set_option("event_timing", 1)
    x.zero_()
    hp.HPCCG(M, b, x, max_iter=120, device=True)
    kt = M.kernel_times()
    launch_s = kt["spmv_ms"] / kt["spmv_launches"] * 1e-3
    q = M.get_option("x_ring") - 1
    side = (16.0 + 8.0 * q) / q * n if M.get_option("x_defer") == 2 else 0.0
    bench_bytes = 8.0 * M.info()["slots"] + 32.0 * n
    bench_frac = (bench_bytes + side) / launch_s / 8e12
    M.close()
    # the same bytes per call
    cli_bytes = float(v["GPU Summary/SPARSEMV compulsory bytes per call"])
    assert abs(cli_bytes - bench_bytes) <= 1e-4 * bench_bytes, (cli_bytes, bench_bytes)  # (printed to 6 digits)
    assert cred > cli_bytes  # 12 nnz + 20 n against 8 B per slot + 32 B per row
    # the same definition: bytes over the CLI's own time per call, against 8 TB/s
    cli_gbs = float(v["GPU Summary/SPARSEMV compulsory GB/s per rank"])
    assert abs(comp - cli_gbs / 8000.0) <= 1e-4 * comp
    # the CLI's figure computed in this process (its definition: the SPARSEMV
    # class time of the device stamps per call, over the same graph-replayed
    # solve shape) against bench.py's, on one placement
    cli_def_here = bench_bytes / (t_g[3] / (it_g + 1)) / 8e12
    assert abs(cli_def_here - bench_frac) <= 0.05 * bench_frac, (cli_def_here, bench_frac)
    # and the CLI's own process against this one
    assert abs(comp - bench_frac) <= 0.25 * bench_frac, (comp, bench_frac)
