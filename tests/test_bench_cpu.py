"""bench.py's N > 1 line on CPU (gloo, world_size 2): the
per-rank records travel to rank 0 through the same all-gather the GPU run
uses (bench.gather_ranks), and the line assembled from them (bench.build_line)
carries the driver's contract keys, the roofline and CPU-baseline objects,
every rank's transport verdicts (peer_auto_ok / pull_auto_ok / proto_auto_ok,
the transport actually used) and the max-over-ranks SpMV launch time with its
compulsory fraction. The measured numbers are synthetic here; the GPU run
fills the same fields."""
import json
import multiprocessing as mp
import os
import socket
import sys

import pytest

from conftest import ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _FakeM:
    def __init__(self, opts):
        self.opts = opts

    def get_option(self, k):
        return self.opts[k]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sys.path.insert(0, ROOT)
        import bench
        transport = {"peer_allreduce": 1, "halo_pull": 2, "rhalo": 1, "fuse_update": 0, "peer_auto_ok": 1,
                     "pull_auto_ok": 1, "proto_auto_ok": 1, "persist_auto_ok": 1, "resident_update": 0,
                     "resident_retries": 0}
        M = _FakeM(transport)
        meas = {"spmv_avg_s": (340.0 + 10.0 * rank) * 1e-6, "local_elapsed": 3.5 + 0.01 * rank,
                "times_acc": [3.5, 0.01, 0.2, 3.0, 0.004, 0.002, 0.0], "niters_total": 499 * 20}
        rt = {"pci_bus_id": "0000:05:00.0", "rccl_nranks": 0}
        ranks = bench.gather_ranks(dist, world, bench.rank_record(None, M, rank, 0, "host", rt, meas))
        if rank == 0:
            class A:
                steps, warmup, max_iter, stencil = 20, 2, 500, 27
            n = 200
            info = {"nrow": n ** 3, "nnz": 213847192, "slots": 216006144}
            full = dict(meas, elapsed=3.52, it=499, step_s=[0.176] * 20, cold_s=0.5, graph_used=1, upd_ms=31.0,
                        upd_n=500, chk=[4e-15, 1e-70, 0], steps=20, event_steps=1, timing_src="synthetic")
            roof = {"bound": "hbm", "achieved": 6000.0, "peak": 8000.0, "unit": "GB/s", "frac": 0.75,
                    "traffic": 2.04e9, "bytes_per_launch": 2.05e9, "avg_launch_us": 340.0}
            cpu = {"value": 12.0, "unit": "CG iterations/s (global-problem iterations x 2 slabs)", "cores": 16,
                   "kind": "reference", "sample": "synthetic"}
            opts = dict(transport, device_bytes=4.2e9, fuse_p=1, fold=1, x_defer=2, x_ring=32, graph_chunk=32, nt=1,
                        a2_ring=3, nt_store=0)
            tchk = bench.rtrans_check([1.0, 0.5, 0.25, 0.125, 0.0625, 0.03125], [1.0, 0.5, 0.25, 0.125, 0.0625,
                                                                                   0.03125], bench.RTRANS_RTOL_MULTI)
            sec = [{"workload": "HPCCG solve, 27-pt 100x100x100 per GPU, z-stacked", "value": 44000.0,
                    "n_gpus": world, "check": {"trace_vs_oracle": tchk}}]
            line = bench.build_line(A, world, n, full, roof, 2, 3, 1, info, opts, dict(rt), ranks, cpu, sec,
                                    {"ran": False}, tchk)
            q.put(json.dumps(line))
        else:
            q.put(None)
    except Exception as e:  # reported to the test
        q.put(json.dumps({"error": repr(e)}))
    finally:
        dist.destroy_process_group()


def test_bench_multirank_line_schema():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    lines = [json.loads(g) for g in got if g is not None]
    assert len(lines) == 1
    d = lines[0]
    assert "error" not in d, d
    # the driver's contract
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["dtype"] == "f64" and d["higher_is_better"] is True
    assert d["value"] == pytest.approx(499 * 20 / 3.52 * 2, rel=1e-6)
    assert d["config"]["workload"].startswith("HPCCG solve, 27-pt 200x200x200 per GPU")
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in d["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in d["cpu_baseline"], k
    # every rank's record, the transport verdicts and the slowest rank's launch
    rk = d["runtime"]["ranks"]
    assert [r["rank"] for r in rk] == [0, 1]
    for r in rk:
        assert r["transport"]["peer_auto_ok"] == 1 and r["transport"]["proto_auto_ok"] == 1
    mr = d["multirank"]
    assert mr["spmv_avg_us_max_over_ranks"] == pytest.approx(350.0) and mr["slowest_rank"] == 1
    assert mr["frac_max_over_ranks"] == pytest.approx(2.05e9 / 350e-6 / 1e9 / 8000.0, rel=1e-3)
    assert mr["transport_used"].startswith("in-kernel")
    assert d["check"]["resident_retries_max_over_ranks"] == 0 and mr["resident_retries_per_rank"] == [0, 0]
    assert len(mr["verdicts_per_rank"]) == 2
    # the N > 1 line checks itself against the oracle and
    # carries north_star's second size (100^3 per GPU)
    tv = d["check"]["trace_vs_oracle"]
    assert tv["ok"] is True and tv["checked"] == 6 and tv["rtol"] == 1e-7
    assert d["secondary"][0]["workload"].startswith("HPCCG solve, 27-pt 100x100x100 per GPU")
    assert d["secondary"][0]["check"]["trace_vs_oracle"]["ok"] is True


class _FakeInfoM(_FakeM):
    def __init__(self, opts, info):
        super().__init__(opts)
        self._info = info

    def info(self):
        return self._info


@pytest.mark.parametrize("ru,kname", [(8, "k_cg_persist"), (1, "k_spmv_ar"), (0, "k_spmv_a")])
def test_roofline_bytes_per_launch_by_resident_mode(ru, kname):
    """bench.roofline_of's compulsory bytes for the 100^3 launch forms: the
    persistent launch (per iteration: 8 B per slot + 32 B per row, no side
    blocks -- x stays in registers -- and no update blocks), k_spmv_ar (side
    blocks, no update blocks), the unit + update-block launch (both)."""
    sys.path.insert(0, ROOT)
    import bench
    n = 100
    nrow, slots = n ** 3, 27012096
    opts = {"spmv_kernel": 1, "a2_ring": 3, "resident_update": ru, "fuse_p": 1, "x_defer": 2, "x_ring": 32,
            "fuse_update": 1, "nt": 0}
    M = _FakeInfoM(opts, {"nrow": nrow, "nnz": 26463592, "slots": slots})
    roof, kernel, kfmt, fused, fupd = bench.roofline_of(M, n, 27, 45e-6)
    assert roof["kernel"].startswith(kname + ":")
    q = 31
    side = (16.0 + 8.0 * q) / q * nrow
    expect = 8.0 * slots + 32.0 * nrow + (0.0 if ru >= 6 else side) + (24.0 * nrow if ru == 0 else 0.0)
    assert roof["bytes_per_launch"] == pytest.approx(expect)
    assert roof["frac"] == pytest.approx(expect / 45e-6 / 1e9 / bench.HBM_PEAK_GBS, rel=1e-3)
    assert ("launch_note" in roof) == (ru >= 6)


def test_rtrans_check():
    """bench.rtrans_check is conftest.check_trace as a record: points above the
    1e-20 cutoff compared on normr^2 at rtol; a miss or too few points fails."""
    sys.path.insert(0, ROOT)
    import bench
    ref = [10.0 ** (-k) for k in range(14)]  # normr; rtrans falls below 1e-20 r0^2 at k = 11
    r = bench.rtrans_check(ref, ref, 1e-7)
    assert r["ok"] and r["checked"] == 11 and r["max_rel"] == 0.0
    bad = list(ref)
    bad[7] *= 1.0 + 1e-7  # rtrans off by 2e-7
    r = bench.rtrans_check(bad, ref, 1e-7)
    assert not r["ok"] and r["first_failing_k"] == 7 and r["max_rel"] == pytest.approx(2e-7, rel=1e-3)
    assert bench.rtrans_check(bad, ref, 1e-6)["ok"]
    assert not bench.rtrans_check(ref[:3], ref, 1e-7)["ok"]  # fewer than TRACE_MIN_POINTS
    assert not bench.rtrans_check([], ref, 1e-7)["ok"]


def test_cpulist_and_no_omp_binding_exported():
    """The job's cpuset parser, and importing bench exports no
    OpenMP binding: a torch.distributed.run started from it would otherwise
    bind every rank to one core."""
    sys.path.insert(0, ROOT)
    env_before = {k: os.environ.get(k) for k in ("OMP_PROC_BIND", "OMP_PLACES")}
    import bench
    assert {k: os.environ.get(k) for k in env_before} == env_before
    assert bench.parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    cpus, src = bench.job_cpuset()
    assert cpus and src


def test_cpu_child_global_problem_and_trace(tmp_path):
    """rank 0's CPU work in a fresh process (bench.py --cpu-child): the mask is
    the job's whole cpuset, threads never exceed its physical cores, the
    reference leg runs on the GLOBAL z-stacked problem of 2 slabs, and the
    OpenMP oracle trace it returns matches the serial oracle's at the multi-
    rank tolerance -- the trace rank 0 checks its GPU trace against."""
    import subprocess
    sys.path.insert(0, ROOT)
    import bench
    import oracle
    spec = {"baseline": {"nx": 16, "ny": 16, "nz": 32, "use_7pt": False, "world": 2, "budget_s": 0.5,
                         "budget_1t_s": 0.5},
            "traces": {"headline": {"nx": 16, "ny": 16, "nz": 32, "use_7pt": False, "iters": 30, "budget_s": 5.0},
                       "secondary0": {"nx": 12, "ny": 12, "nz": 24, "use_7pt": True, "iters": 30, "budget_s": 5.0}}}
    sp, op = tmp_path / "spec.json", tmp_path / "out.json"
    sp.write_text(json.dumps(spec))
    env = {k: v for k, v in os.environ.items() if not k.startswith("OMP_")}
    subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-child", str(sp), str(op)], check=True,
                   env=env, stdout=subprocess.DEVNULL, timeout=240)
    out = json.loads(op.read_text())
    m = out["mask"]
    cpus, _ = bench.job_cpuset()
    assert m["cpus"] == len(cpus & set(range(os.cpu_count())))
    assert 1 <= m["threads"] <= m["physical_cores"]
    base = out["baseline"]
    assert "error" not in base, base
    if oracle.ref_available():
        assert base["kind"] == "reference" and base["leg"] == "host" and base["cores"] == m["threads"]
        assert base["sample"].startswith("global 16x16x32 (the 2 slabs together)")
        assert base["value"] == pytest.approx(2 * base["global_iterations_per_s"])
    for name, (nx, nz, s7) in {"headline": (16, 32, False), "secondary0": (12, 24, True)}.items():
        tr = out["traces"][name]
        assert tr["iterations"] == 30 and len(tr["trace"]) == 31
        serial = oracle.hpccg(oracle.generate(nx, nx, nz, use_7pt=s7), max_iter=31)["trace"]
        chk = bench.rtrans_check(tr["trace"], serial, bench.RTRANS_RTOL_MULTI)
        assert chk["ok"], chk
