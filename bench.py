#!/usr/bin/env python3
"""bench.py -- HPCCG on MI355X: CG iterations/s and effective SpMV GB/s.

One *step* = one full HPCCG() solve (HPCCG.cpp:312-402) with max_iter = 500
(499 CG iterations, tolerance 0: main.cpp:187-188) on the 27-point
nx = ny = nz = 200 problem per GPU (BASELINE.json configs[2]), matrix, b and
x resident in HBM before the timed region (device generator).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 200] [--stencil 27]

N > 1: one process per rank under torch.distributed.run (the driver's launch;
`python bench.py --gpus N` without WORLD_SIZE starts that launcher itself as a
child process before touching a GPU); z-stacked slabs (local nz fixed, weak
scaling). One rank per GPU over RCCL (--comm rccl, the default when there are
at least N GPUs): after the creation-time self-tests the iteration sums its two
scalars inside the kernels and pulls its ghost planes from the neighbours'
memory, RCCL being the fallback; with fewer GPUs than ranks (--comm host) the
ranks share GPUs and bootstrap through the host (hpccg_hip_comm_init_host),
running the same in-kernel transport between processes. torch.distributed
(gloo) carries only the control plane (unique id / setup all-gathers, barrier,
max-over-ranks time). The line carries every rank's transport verdicts, the
max-over-ranks SpMV launch time, and a CPU leg on the global problem.

value = (CG iterations x ranks x K) / max-over-ranks wall time of the K steps
      = 200^3-slab CG iterations per second summed over GPUs.
roofline (the SpMV kernel, 84 % of the reference's time):
  achieved = the bytes the SpMV must move in its matrix format (values of the
  SELL-512-A image, 8 B per stored slot incl. holes, + the vectors it reads
  and writes once) per launch / the average launch time from hipEvents on the
  solver stream in the first --event-steps timed steps (eager; the other
  steps replay hipGraphs); frac = achieved / 8 TB/s (MI355X HBM3E spec);
  frac_vs_copy_ceiling against the measured 6.29 TB/s float4 copy
  (MI355X_MICROARCH.md). traffic = HBM bytes per launch from the committed
  rocprofv3 FETCH_SIZE / WRITE_SIZE passes of the same kernel
  (profiles/pmc_spmv_<stencil>pt_<n>.json), or null. credited_frac keeps
  SURVEY 8(d)'s fixed formula (12 nnz + 20 n SpMV + ddot/waxpby bytes the
  fused kernel absorbs) is reported as bytes only.
cpu_baseline: the reference compiled from its own sources (oracle/_ref) on
  a bounded sample of the same problem, run by rank 0 after every GPU step in
  a fresh child process (`bench.py --cpu-child`) whose CPU mask is widened to
  the job's whole cpuset (cgroup cpuset.cpus.effective) before any OpenMP
  runtime loads -- never the launched rank's own, possibly narrowed, mask.
  Legs: the OpenMP build with one thread per physical core of that mask,
  capped by the cgroup CPU quota (the host bar), the OpenMP build with the
  box's thread share (OMP_NUM_THREADS) when that differs, and (N = 1) the
  serial build; value = the fastest leg, cores = its thread count. N > 1: the
  reference on the global nx x ny x (N nz) problem; value in
  the same unit as the line's (global-problem iterations/s x N, i.e.
  per-GPU-slab iterations summed).
check.trace_vs_oracle: the same child runs the oracle (oracle/hpccg_oracle.c,
  pinned to the reference) on the GLOBAL problem for its first iterations and
  rank 0 compares its GPU rtrans trace point by point above the 1e-20 cutoff
  (tests/conftest.py's stated tolerance: 1e-8 on one rank, 1e-7 over ranks);
  a failed check makes the run exit 3 after the line is printed.
secondary: the other configs of BASELINE.json measured in the same run the
  same way -- N = 1: 27-pt 100^3 and 7-pt 256^3; N > 1: 27-pt 100^3 per GPU,
  weak-scaled like the headline (north_star's second size at 1/2/4/8 GPUs):
  value, launch time, compulsory-byte fraction, committed PMC traffic ratio,
  its own trace check; no CPU leg.
host_boundary (N = 1): the rate a caller of the reference's own HPCCG()
  interface sees -- the C drop-in hpccg_hip_HPCCG on a host HPC_Sparse_Matrix
  with host b and x (PCIe copies included; the device image cached by a first,
  untimed call); informational, never value.

Multi-GPU runs describe themselves: every rank logs its stages on stderr
(comm init, setup, first solve, timed steps), the line carries what RCCL
reports (ncclCommCount, versions, the loaded RCCL / HIP objects, every rank's
PCI bus id) and the per-iteration halo / all-reduce time, and a watchdog ends
a rank (exit 124) whose run outlives --timeout; the parent that starts
torch.distributed.run kills the job at the same limit.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

# This process's CPU mask at start-up, for the record only: the CPU legs run
# in a child that widens its own mask (cpu_child). No OpenMP binding variables
# are set here: exported into the environment they would make torch's libgomp
# bind this process -- and a torch.distributed.run launched from it, and so
# every rank -- to a single core.
AFFINITY_MASK = sorted(os.sched_getaffinity(0))
AFFINITY_CPUS = len(AFFINITY_MASK)

ROOT = os.path.dirname(os.path.abspath(__file__))
# tests/conftest.py's stated fp64 parity tolerance on rtrans = normr^2
RTRANS_RTOL_1GPU = 1e-8
RTRANS_RTOL_MULTI = 1e-7
RTRANS_CUTOFF = 1e-20
TRACE_MIN_POINTS = 5
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
COPY_CEILING_GBS = 6290.0  # MI355X_MICROARCH.md: float4 copy, measured
KERNEL_NAMES = {0: "k_spmv_sell", 1: "k_spmv_a", 2: "k_spmv_a2", 3: "k_spmv_a2r", 4: "k_spmv_ar", 5: "k_cg_persist"}
FORMAT_NAMES = {0: "SELL-512 (8 B value + 4 B int32 column per slot)",
                1: "SELL-512-A (8 B value per offset-aligned slot, holes 0.0), x read at the slice's offsets",
                2: "SELL-512-A (8 B value per offset-aligned slot, holes 0.0), x from LDS windows shared by slice "
                   "pairs",
                3: "SELL-512-A (8 B value per offset-aligned slot, holes 0.0), x from LDS windows shared by slice "
                   "pairs, values streamed HBM -> LDS by per-wave LDS-DMA rings",
                4: "SELL-512-A (8 B value per offset-aligned slot, holes 0.0), x read at the slice's offsets, one "
                   "block per slice pair, every block resident: the update applied from registers (no Ap stream)",
                5: "SELL-512-A (8 B value per offset-aligned slot, holes 0.0), x read at the slice's offsets, one "
                   "block per slice pair, every block resident for the whole solve: one launch runs every "
                   "iteration, x and the update in registers"}


def load_pkg():
    import importlib.util
    name = "hpccg_sycl_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "hpccg-sycl_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cpu(mask=None):
    """CPU model and counts of the host (lscpu), the CPU mask the legs ran on
    and the one this (launched) process started with."""
    info = {"affinity_cpus": len(mask) if mask is not None else AFFINITY_CPUS,
            "launch_affinity_cpus": AFFINITY_CPUS,
            "omp_proc_bind": os.environ.get("OMP_PROC_BIND"), "omp_places": os.environ.get("OMP_PLACES")}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k in ("Model name", "CPU(s)", "Socket(s)", "Core(s) per socket", "Thread(s) per core"):
                info[k] = v
    except Exception as e:  # reported, not fatal
        info["lscpu_error"] = repr(e)
    q = cgroup_quota()
    if q is not None:
        info["cgroup_cpu_max"] = q[0]
        if q[1] is not None:
            info["cgroup_cpu_quota_cores"] = round(q[1], 2)
    return info


def cgroup_quota():
    """The cgroup v2 CPU bandwidth quota ("quota period", cores or None when
    unlimited): on a shared box it, not the affinity mask, bounds how many
    threads run at once. None when the file is absent."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
    except (OSError, ValueError):
        return None
    return f"{q} {per}", (None if q == "max" else int(q) / int(per))


def parse_cpulist(txt):
    """'0-3,8,10-11' -> {0, 1, 2, 3, 8, 10, 11}."""
    cpus = set()
    for part in txt.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
    return cpus


def job_cpuset():
    """The CPUs the job's cgroup may use (cpuset.cpus.effective), else every
    online CPU."""
    for p in ("/sys/fs/cgroup/cpuset.cpus.effective", "/sys/fs/cgroup/cpuset/cpuset.effective_cpus"):
        try:
            with open(p) as f:
                cpus = parse_cpulist(f.read())
            if cpus:
                return cpus, p
        except (OSError, ValueError):
            continue
    try:
        with open("/sys/devices/system/cpu/online") as f:
            return parse_cpulist(f.read()), "/sys/devices/system/cpu/online"
    except (OSError, ValueError):
        return set(range(os.cpu_count() or 1)), "os.cpu_count()"


def physical_cores(mask):
    """Physical cores (distinct package/core ids) among the CPUs of `mask`."""
    cores = set()
    for c in mask:
        t = f"/sys/devices/system/cpu/cpu{c}/topology"
        try:
            with open(f"{t}/physical_package_id") as f1, open(f"{t}/core_id") as f2:
                cores.add((f1.read().strip(), f2.read().strip()))
        except OSError:
            cores.add(("?", str(c)))
    return len(cores)


def host_threads(mask):
    """One OpenMP thread per physical core of `mask`, capped by the cgroup CPU
    quota (more threads than the quota's cores only time-slice)."""
    phys = physical_cores(mask)
    q = cgroup_quota()
    if q is not None and q[1] is not None:
        return max(1, min(phys, int(q[1]))), phys
    return max(1, phys), phys


def rtrans_check(gpu_tr, ref_tr, rtol):
    """tests/conftest.py check_trace as a record: every k with
    rtrans_ref,k >= 1e-20 rtrans_ref,0 (rtrans = normr^2) compared at `rtol`;
    ok when no point exceeds it and at least TRACE_MIN_POINTS were compared."""
    g = [float(v) for v in gpu_tr]
    r = [float(v) for v in ref_tr]
    if not g or not r:
        return {"checked": 0, "max_rel": None, "rtol": rtol, "ok": False, "note": "empty trace"}
    r0 = r[0] ** 2
    checked, max_rel, first_bad = 0, 0.0, None
    for k in range(min(len(g), len(r))):
        rr = r[k] ** 2
        if rr < RTRANS_CUTOFF * r0:
            break
        rel = abs(g[k] ** 2 - rr) / rr if rr > 0 else abs(g[k] ** 2)
        if rel > rtol and first_bad is None:
            first_bad = k
        max_rel = max(max_rel, rel)
        checked += 1
    return {"checked": checked, "max_rel": max_rel, "rtol": rtol, "first_failing_k": first_bad,
            "ok": first_bad is None and checked >= TRACE_MIN_POINTS}


def _ref_legs(oracle, A, legs, nx, ny, nz, use_7pt, world):
    """The reference's HPCCG() (oracle/_ref) on `A`, one bounded solve per
    leg (the first iterations of it, sized by a 3-iteration probe)."""
    import ctypes
    gomp = ctypes.CDLL("libgomp.so.1") if os.path.exists(oracle.REF_OMP_SO) else None  # the ref build's runtime
    out = {}
    mats = {}
    saved = os.dup(1)  # the reference prints its residual lines on fd 1
    null = os.open(os.devnull, os.O_WRONLY)
    os.dup2(null, 1)
    try:
        for leg, nthreads, budget in legs:
            omp = leg != "serial"
            if omp:
                gomp.omp_set_num_threads(nthreads)
            if omp not in mats:
                mats[omp] = oracle.ref_from_csr(A, omp=omp)
            M = mats[omp]
            probe = 2 if world > 1 else 3
            t = oracle.ref_hpccg(M, A.b, max_iter=probe + 1)["times"][0]
            iters = int(max(probe, min(500, budget / max(t / probe, 1e-6))))
            res = oracle.ref_hpccg(M, A.b, max_iter=iters + 1)
            its = res["niters"] / max(res["times"][0], 1e-9)  # (a tiny sample can round to 0 s)
            what = (f"global {nx}x{ny}x{nz} (the {world} slabs together)" if world > 1 else f"{nx}x{ny}x{nz}")
            sample = (f"{what} {'7' if use_7pt else '27'}-pt, first {res['niters']} CG iterations of one reference "
                      f"HPCCG() solve ({res['times'][0]:.1f} s)")
            desc = (f", OpenMP {nthreads} threads (OMP_PROC_BIND={os.environ.get('OMP_PROC_BIND')}, "
                    f"OMP_PLACES={os.environ.get('OMP_PLACES')})" if omp else ", serial")
            out[leg] = {"value": its * world, "global_iterations_per_s": its, "threads": nthreads,
                        "kind": "reference", "sample": sample + desc}
    finally:
        ctypes.CDLL(None).fflush(None)
        os.dup2(saved, 1)
        os.close(null)
        os.close(saved)
        for M in mats.values():
            M.close()
    return out


def _oracle_trace(oracle, A, nthreads, iters, budget_s):
    """The oracle's HPCCG() (hpccg_oracle.c: HPCCG.cpp:312-402 restated,
    pinned to the reference) on `A`: the rtrans trace of its first iterations
    (at most `iters`, fewer when a 2-iteration probe says the budget is short)."""
    t0 = time.perf_counter()
    oracle.hpccg(A, max_iter=3, nthreads=nthreads, trace=False)
    per_it = max((time.perf_counter() - t0) / 2, 1e-6)
    k = int(max(TRACE_MIN_POINTS + 2, min(iters, budget_s / per_it)))
    t0 = time.perf_counter()
    res = oracle.hpccg(A, max_iter=k + 1, nthreads=nthreads, trace=True)
    return {"trace": [float(v) for v in res["trace"]], "iterations": res["niters"],
            "seconds": round(time.perf_counter() - t0, 2), "threads": nthreads}


def cpu_child(spec_path, out_path):
    """`bench.py --cpu-child SPEC OUT`: rank 0's CPU work, in a fresh process
    that has touched no GPU. The mask is widened to the job's cpuset before
    any OpenMP runtime loads; then the reference's legs on the baseline
    problem and the oracle's traces of the listed (global) problems; the
    result goes to OUT as JSON."""
    with open(spec_path) as f:
        spec = json.load(f)
    launch_mask = sorted(os.sched_getaffinity(0))
    want, src = job_cpuset()
    try:
        os.sched_setaffinity(0, want)
    except OSError as e:
        log(f"cpu-child: could not widen the CPU mask to {src}: {e!r}")
    mask = sorted(os.sched_getaffinity(0))
    threads, phys = host_threads(mask)
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    # before libgomp loads (the oracle and the reference build both use it)
    os.environ.update(OMP_NUM_THREADS=str(threads), OMP_PROC_BIND="spread", OMP_PLACES="cores")
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the baseline leg and the trace check only
    result = {"mask": {"launch_cpus": len(launch_mask), "cpus": len(mask), "cpuset_source": src,
                       "physical_cores": phys, "threads": threads}, "traces": {}}
    cache = {}

    def problem(nx, ny, nz, use_7pt):
        key = (nx, ny, nz, use_7pt)
        if key not in cache:
            cache.clear()  # one global problem in memory at a time
            cache[key] = oracle.generate(nx, ny, nz, use_7pt=use_7pt)
        return cache[key]

    base = spec.get("baseline")
    if base:
        t0 = time.time()
        try:
            A = problem(base["nx"], base["ny"], base["nz"], base["use_7pt"])
            setup_s = time.time() - t0
            world = base["world"]
            legs = []
            if os.path.exists(oracle.REF_OMP_SO):
                legs.append(("host", threads, base["budget_s"]))
                if share and share != threads:
                    legs.append(("box_share", share, base["budget_s"]))
            if world == 1 and os.path.exists(oracle.REF_SO):
                legs.append(("serial", 1, base["budget_1t_s"]))
            if not legs:
                raise RuntimeError("oracle/_ref is not built (make -C oracle ref)")
            out = {"unit": "CG iterations/s" if world == 1 else
                   "CG iterations/s (global-problem iterations x %d slabs)" % world,
                   "legs": _ref_legs(oracle, A, legs, base["nx"], base["ny"], base["nz"], base["use_7pt"], world),
                   "host": host_cpu(mask), "setup_s": round(setup_s, 1)}
            out["host"]["physical_cores_in_affinity"] = phys
            out["host"]["cpuset_source"] = src
            best_leg = max(out["legs"], key=lambda k: out["legs"][k]["value"])
            best = out["legs"][best_leg]
            out.update({"value": best["value"], "cores": best["threads"], "threads": best["threads"],
                        "physical_cores": phys, "kind": "reference", "leg": best_leg, "sample": best["sample"]})
            if world > 1:
                out["global_iterations_per_s"] = best["global_iterations_per_s"]
            if "serial" in out["legs"]:
                s = out["legs"]["serial"]
                out["single_thread"] = {"value": s["value"], "cores": 1, "kind": "reference", "sample": s["sample"]}
            assert out["physical_cores"] >= out["threads"] or best_leg == "box_share", out
            result["baseline"] = out
        except Exception as e:  # reported, never silently replaced
            result["baseline"] = {"error": repr(e)}
    for name, tj in spec.get("traces", {}).items():
        try:
            A = problem(tj["nx"], tj["ny"], tj["nz"], tj["use_7pt"])
            result["traces"][name] = _oracle_trace(oracle, A, threads, tj["iters"], tj["budget_s"])
        except Exception as e:
            result["traces"][name] = {"error": repr(e)}
        log(f"cpu-child: trace {name} done")
    with open(out_path, "w") as f:
        json.dump(result, f)


def run_cpu_child(spec, timeout_s):
    """Rank 0: run cpu_child in a fresh process (a child, not an exec: this
    process has initialised the GPU) and return its JSON, or {"error": ...}."""
    import tempfile
    with tempfile.TemporaryDirectory(prefix="hpccg_cpu_") as d:
        sp, op = os.path.join(d, "spec.json"), os.path.join(d, "out.json")
        with open(sp, "w") as f:
            json.dump(spec, f)
        env = {k: v for k, v in os.environ.items() if k not in ("OMP_PROC_BIND", "OMP_PLACES")}
        t0 = time.time()
        try:
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-child", sp, op],
                               stdout=subprocess.DEVNULL, env=env, timeout=timeout_s)
        except subprocess.TimeoutExpired:
            return {"error": f"cpu child exceeded {timeout_s:.0f} s"}
        if p.returncode != 0 or not os.path.exists(op):
            return {"error": f"cpu child exited {p.returncode}"}
        with open(op) as f:
            out = json.load(f)
        out["seconds"] = round(time.time() - t0, 1)
        return out


def pmc_traffic(tag, kernel, fused, xdefer, fupd, resident=0):
    """HBM bytes per SpMV launch from the committed rocprofv3 FETCH/WRITE
    passes of the same kernel configuration (profiles/pmc_<tag>.json; matched
    by kernel template name, fusion and x deferral), else (None, None)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{tag}.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    name = d.get("kernel", "")
    if KERNEL_NAMES[kernel] + "<" not in name or bool(d.get("fuse_p")) != bool(fused) or \
            d.get("x_defer", 1) != xdefer or d.get("fuse_update", 0) != fupd or d.get("resident_update", 0) != resident:
        return None, None
    return d.get("spmv_hbm_bytes_per_launch"), f"profiles/pmc_{tag}.json ({d.get('tag', '?')}), matched by kernel name"


def placement_report(tries, probe_us, pick):
    """The placement probe only when asked for (--placement):
    the creation placement's and the kept placement's CG iteration time as
    separate fields, so the gain is visible and never folded into value
    unannounced."""
    if not len(probe_us):
        return {"ran": False, "requested": tries}
    us = [float(v) for v in probe_us]
    creation, kept = us[0], min(us)
    return {"ran": True, "requested": tries,
            "note": "setup, untimed: CG iterations timed on candidate placements (plain allocations) of the values, the "
                    "p ring, r and Ap, fastest kept; rank 0's",
            "creation_us_per_iteration": round(creation, 2), "kept_us_per_iteration": round(kept, 2),
            "gain_frac": round(creation / kept - 1.0, 4),
            "us_per_iteration": [round(v, 2) for v in us],
            "kept": {b: (pick >> (8 * i)) & 255 for i, b in enumerate(("values", "ring", "r", "Ap"))}}


def relaunch_distributed(args):
    """--gpus N > 1 without a launcher: start torch.distributed.run as a child
    (nothing has touched the GPU yet) and exit with its code; past --timeout
    the whole job (its own process group) is killed and the exit code is 124."""
    import signal
    port = 29400 + (os.getpid() % 500)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    log("launching:", " ".join(cmd))
    p = subprocess.Popen(cmd, env=env, start_new_session=True)
    try:
        return p.wait(timeout=args.timeout)
    except subprocess.TimeoutExpired:
        log(f"bench: job exceeded --timeout {args.timeout:.0f} s; killing process group {p.pid}")
        os.killpg(p.pid, signal.SIGTERM)
        try:
            p.wait(timeout=20)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
        return 124


class Stages:
    """Per-rank progress on stderr, and a watchdog: a rank whose run outlives
    the limit reports the stage it is stuck in and exits (124) instead of
    leaving a hung job that records nothing."""

    def __init__(self, rank, limit_s):
        import threading
        self.rank, self.t0, self.stage = rank, time.time(), "start"
        self.done = threading.Event()
        threading.Thread(target=self._watch, args=(limit_s if limit_s > 0 else float("inf"),), daemon=True).start()

    def __call__(self, stage, **kv):
        self.stage = stage
        extra = " ".join(f"{k}={v}" for k, v in kv.items())
        log(f"[rank {self.rank}] +{time.time() - self.t0:7.2f}s {stage} {extra}".rstrip())

    def _watch(self, limit_s):
        # a heartbeat every 30 s (a long stage -- 8 ranks sharing one GPU, the
        # CPU child on a global problem -- must not look hung), then the limit
        t_end = self.t0 + limit_s
        while not self.done.wait(min(30.0, max(0.0, t_end - time.time()))):
            if time.time() >= t_end:
                log(f"[rank {self.rank}] watchdog: still in stage '{self.stage}' after {limit_s:.0f} s; exiting 124")
                os._exit(124)
            if self.rank == 0:
                log(f"[rank {self.rank}] +{time.time() - self.t0:7.2f}s ... in stage '{self.stage}'")


def init_gloo(dist, rank, world):
    """torch.distributed's gloo group for the control plane. Gloo prints its
    connection banner on fd 1: kept off stdout, which carries one JSON line."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dist.barrier()
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def opt_or_none(M, key):
    """An option's effective value, or None where the library predates it."""
    try:
        return M.get_option(key)
    except Exception:
        return None


def measure(hp, torch, M, dev, max_iter, steps, warmup, event_steps, world, dist=None, stage=None):
    """Warmup, then `steps` timed solves bracketed by a barrier and a device
    sync on both sides; the first `event_steps` of them eager with hipEvents
    around every SpMV launch (the roofline's kernel time), the rest graph
    replays. Returns the raw numbers (elapsed is the max over ranks)."""
    b, _, _ = M.vectors()
    nrow = M.info()["nrow"]
    x = torch.zeros(nrow, dtype=torch.float64, device=f"cuda:{dev}")
    torch.cuda.synchronize()

    def step(events):
        M.set_option("event_timing", 1 if events else 0)
        x.zero_()
        return hp.HPCCG(M, b, x, max_iter=max_iter, device=True)

    def barrier():
        if world > 1:
            dist.barrier()

    cold_s = None
    # the ranks start their first solve together: its in-kernel waits for the
    # other ranks' contributions are bounded (spin_budget_us), so setup skew
    # between ranks must not eat into them
    barrier()
    for i in range(warmup):
        t0 = time.perf_counter()
        step(i == 0)
        if i == 0:
            cold_s = time.perf_counter() - t0  # first solve: graph build, cold caches
            if stage:
                stage("first_solve", seconds=f"{cold_s:.3f}")
    barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    niters_total = 0
    spmv_ms = spmv_n = upd_ms = upd_n = 0.0
    times_acc = [0.0] * 7
    step_s = []
    graph_used = 1
    it, nr = 0, 0.0
    for i in range(steps):
        ev = i < event_steps
        t0 = time.perf_counter()
        _, it, nr, times = step(ev)
        step_s.append(time.perf_counter() - t0)
        niters_total += it
        if ev:
            kt = M.kernel_times()
            spmv_ms += kt["spmv_ms"]
            spmv_n += kt["spmv_launches"]
            upd_ms += kt["update_ms"]
            upd_n += kt["update_launches"]
        else:
            graph_used = min(graph_used, M.get_option("graph_used"))
        for j in range(7):
            times_acc[j] += times[j]
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t_start
    local_elapsed = elapsed
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    # outside the timed region: the last solve's answer (xexact = 1, generate_matrix.cpp:286)
    # and residual reduction, max over ranks -- a wrong multi-rank exchange shows here
    tr = M.last_trace()
    # resident launches re-run after an expired wait (none expected on a box of our own)
    retries = opt_or_none(M, "resident_retries") or 0
    chk = torch.tensor([(x - 1.0).abs().max().item(), float(nr / tr[0]) if tr[0] > 0 else 0.0, float(retries)],
                       dtype=torch.float64)
    if world > 1:
        dist.all_reduce(chk, op=dist.ReduceOp.MAX)
    if spmv_n > 0:
        spmv_avg_s = spmv_ms / spmv_n * 1e-3
        timing_src = ("hipEvent pairs around every SpMV launch on the solver stream, %d of the %d timed steps "
                      "(eager; the others replay hipGraphs)" % (event_steps, steps))
    else:  # graph mode only: device-clock stamps (SPARSEMV class time / calls)
        spmv_avg_s = times_acc[3] / max(1, niters_total + steps)
        timing_src = "s_memrealtime stamps (graph mode)"
    return {"elapsed": elapsed, "local_elapsed": local_elapsed, "niters_total": niters_total, "it": it,
            "spmv_avg_s": spmv_avg_s, "timing_src": timing_src, "upd_ms": upd_ms, "upd_n": upd_n,
            "times_acc": times_acc, "step_s": step_s, "cold_s": cold_s, "graph_used": graph_used,
            "chk": [chk[0].item(), chk[1].item(), int(chk[2].item())], "steps": steps, "event_steps": event_steps,
            "trace": [float(v) for v in tr]}


def roofline_of(M, n, stencil, spmv_avg_s):
    """The SpMV launch against the HBM roofline: format-compulsory bytes
     over the launch time, the committed PMC traffic of the same
    kernel configuration, SURVEY 8(d)'s credited bytes beside them."""
    info = M.info()
    nrow = info["nrow"]
    kernel = M.get_option("spmv_kernel")
    kfmt = 3 if (kernel == 2 and M.get_option("a2_ring") > 0) else kernel  # 3: the pair kernel's LDS-DMA ring form
    ru = opt_or_none(M, "resident_update") or 0
    resident = ru >= 1
    persist = ru >= 6  # one launch per solve (k_cg_persist): the figures are per iteration of it
    if resident:
        kfmt = 5 if persist else 4  # the resident pair kernel (k_spmv_ar)
    fused = M.get_option("fuse_p")
    slots = info["slots"]
    # bytes the SpMV must move in its format: the stored slots (8 B; SELL-512
    # also 4 B of column), p or (r, p_{k-1}) once, p_k and Ap written
    slot_bytes = 12.0 if kernel == 0 else 8.0
    vec_bytes = (32.0 if fused else 16.0) * nrow
    # x_defer 2: the launch's trailing blocks apply the deferred x terms of
    # 1/q of the rows (q = x_ring - 1): x read and written, q p's read
    xside = M.get_option("x_defer") == 2 and not persist  # (persistent: x stays in registers)
    q = M.get_option("x_ring") - 1
    side_bytes = (16.0 + 8.0 * q) / q * nrow if xside else 0.0
    # fused update: the launch's trailing blocks also run the update (r, Ap read; r written);
    # resident: the units apply it from registers -- r written instead of Ap, nothing read back
    fupd = M.get_option("fuse_update") == 1
    upd_bytes = 24.0 * nrow if (fupd and not resident) else 0.0
    format_bytes = slot_bytes * slots + vec_bytes + side_bytes + upd_bytes
    # SURVEY 8(d) credited bytes: HPC_sparsemv 12 nnz + 20 n, ddot(p, Ap) 16 n,
    # with the fused p update the waxpby p = r + beta p, 24 n
    credited = 12.0 * info["nnz"] + 20.0 * nrow + 16.0 * nrow + (24.0 * nrow if fused else 0.0)
    achieved = format_bytes / spmv_avg_s / 1e9
    traffic, traffic_src = pmc_traffic(f"spmv_{stencil}pt_{n}", kfmt, fused, M.get_option("x_defer"),
                                       M.get_option("fuse_update"), ru if resident else 0)
    roof = {
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "traffic_source": traffic_src,
        # FETCH_SIZE / WRITE_SIZE count the L2 <-> fabric bytes: Infinity
        # Cache (MALL) hits are in them. An image under 256 MB (100^3)
        # may be served partly by the MALL, so "hbm" is its upper bound.
        "traffic_note": "L2-fabric bytes (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE), Infinity Cache hits included",
        "traffic_over_compulsory": round(traffic / format_bytes, 4) if traffic else None,
        "image_fits_infinity_cache": not bool(M.get_option("nt")),
        "frac_vs_copy_ceiling": round(achieved / COPY_CEILING_GBS, 4),
        "kernel": "%s: %s + p.Ap%s" % (KERNEL_NAMES[kfmt], FORMAT_NAMES[kfmt], " + p = r + beta p" if fused else ""),
        "bytes_per_launch": format_bytes,
        "bytes_formula": ("%g B per stored slot x %d slots + 32 B per row (r, p_{k-1} read; p_k, r "
                          "written; Ap%s and the update stay in registers)" % (slot_bytes, slots, ", x" if persist else "")
                          if resident else
                          "%g B per stored slot x %d slots + %d B per row (r, p_{k-1} read; p_k, Ap "
                          "written)" % (slot_bytes, slots, 32) if fused else
                          "%g B per stored slot x %d slots + 16 B per row (p read, Ap written)" % (slot_bytes, slots)) +
                         (" + (16 + 8 q) / q B per row, q = %d (side blocks: x read and written, q p's read "
                          "for 1/q of the rows)" % q if xside else "") +
                         (" + 24 B per row (fused update blocks: r and Ap read, r written)"
                          if (fupd and not resident) else ""),
        # SURVEY 8(d)'s fixed byte formula for the unfused reference sequence
        # this launch replaces (more bytes than this format moves; no rate is
        # derived from it: `frac` above is the roofline fraction)
        "credited_bytes_per_launch": credited,
        "avg_launch_us": round(spmv_avg_s * 1e6, 2),
    }
    if persist:
        roof["launch_note"] = ("one k_cg_persist launch runs every iteration: avg_launch_us is (prologue SpMV + that "
                               "launch) / (iterations + 1), bytes_per_launch one iteration's")
    if traffic:
        roof["traffic_gbs"] = round(traffic / spmv_avg_s / 1e9, 1)
        roof["traffic_frac"] = round(traffic / spmv_avg_s / 1e9 / HBM_PEAK_GBS, 4)
    return roof, kernel, kfmt, fused, fupd


TRANSPORT_KEYS = ("peer_allreduce", "halo_pull", "rhalo", "fuse_update", "peer_auto_ok", "pull_auto_ok",
                  "proto_auto_ok", "persist_auto_ok", "resident_update", "resident_retries")


def rank_record(hp, M, rank, dev, comm_mode, rt, meas):
    """What every rank contributes to the line (gathered to rank 0)."""
    return {"rank": rank, "device": dev, "pci_bus_id": rt.get("pci_bus_id"), "comm": comm_mode,
            "rccl_nranks": rt.get("rccl_nranks"),
            "transport": {k: opt_or_none(M, k) for k in TRANSPORT_KEYS},
            "spmv_avg_us": round(meas["spmv_avg_s"] * 1e6, 3), "local_elapsed_s": round(meas["local_elapsed"], 6),
            "halo_us_per_iteration": round(meas["times_acc"][5] / max(1, meas["niters_total"]) * 1e6, 3),
            "allreduce_us_per_iteration": round(meas["times_acc"][4] / max(1, meas["niters_total"]) * 1e6, 3)}


def gather_ranks(dist, world, rec):
    """Every rank's record, in rank order (gloo)."""
    if world == 1:
        return [rec]
    out = [None] * world
    dist.all_gather_object(out, rec)
    return out


def multirank_summary(ranks, bytes_per_launch):
    """N > 1: the slowest rank's SpMV launch (hipEvents) against the roofline,
    and the transport every rank actually ran."""
    worst = max(ranks, key=lambda r: r["spmv_avg_us"])
    ach = bytes_per_launch / (worst["spmv_avg_us"] * 1e-6) / 1e9
    tr = [r["transport"] for r in ranks]
    in_kernel = all(t.get("peer_allreduce") == 1 and t.get("halo_pull") in (1, 2) for t in tr)
    persistent = all(t.get("resident_update") == 8 for t in tr)
    return {"spmv_avg_us_max_over_ranks": worst["spmv_avg_us"], "slowest_rank": worst["rank"],
            "frac_max_over_ranks": round(ach / HBM_PEAK_GBS, 4),
            "spmv_avg_us_per_rank": [r["spmv_avg_us"] for r in ranks],
            "transport_used": ("in-kernel: peer all-reduce + halo pull inside one persistent launch per solve"
                               if (in_kernel and persistent) else
                               "in-kernel: peer all-reduce + halo pull (no collective call per iteration)"
                               if in_kernel else "RCCL (all-reduce and/or send/recv per iteration) on some rank"),
            "verdicts_per_rank": [{k: t.get(k) for k in ("peer_auto_ok", "pull_auto_ok", "proto_auto_ok",
                                                         "persist_auto_ok")} for t in tr],
            "resident_retries_per_rank": [t.get("resident_retries") for t in tr],
            "halo_us_per_iteration_per_rank": [r["halo_us_per_iteration"] for r in ranks],
            "allreduce_us_per_iteration_per_rank": [r["allreduce_us_per_iteration"] for r in ranks]}


def secondary_config(hp, torch, n, stencil, dev, args, world=1, dist=None, rank=0, comm="none", rt=None):
    """One other config of BASELINE.json, measured like the headline (N > 1:
    n^3 per GPU, z-stacked, every rank takes part)."""
    M = hp.Matrix.generate(n, n, n, use_7pt=stencil == 7)
    try:
        meas = measure(hp, torch, M, dev, args.max_iter, args.secondary_steps, 2, 1, world, dist)
        roof, kernel, kfmt, fused, fupd = roofline_of(M, n, stencil, meas["spmv_avg_s"])
        ranks = gather_ranks(dist, world, rank_record(hp, M, rank, dev, comm, rt or {}, meas))
        value = meas["niters_total"] / meas["elapsed"] * world
        out = {"metric": f"CG iterations/sec + effective SpMV GB/s (% HBM peak), {stencil}-pt nx=ny=nz={n}",
               "workload": f"HPCCG solve, {stencil}-pt {n}x{n}x{n}" + (" per GPU, z-stacked" if world > 1 else "") +
                           f", max_iter={args.max_iter}, tolerance 0",
               "value": round(value, 3),
               "unit": "CG iterations/s" if world == 1 else
                       "CG iterations/s (per-GPU %d^3 slab iterations, summed over GPUs)" % n,
               "n_gpus": world, "scaling": "weak", "steps": meas["steps"],
               "ms_per_step": round(meas["elapsed"] / meas["steps"] * 1e3, 3),
               "avg_launch_us": roof["avg_launch_us"], "frac": roof["frac"],
               "traffic_over_compulsory": roof["traffic_over_compulsory"], "roofline": roof,
               "spmv_kernel": kernel, "graph_replay": bool(meas["graph_used"]),
               "check": {"x_minus_xexact_inf": meas["chk"][0], "final_normr_over_initial": meas["chk"][1],
                         "niters_per_solve": meas["it"], "resident_retries_max_over_ranks": meas["chk"][2]},
               "cpu_baseline": None,
               "cpu_note": "no CPU leg for secondary configs (the headline line carries the reference's)"}
        if world > 1:
            out["multirank"] = multirank_summary(ranks, roof["bytes_per_launch"])
        return out, meas["trace"]
    finally:
        M.close()


def host_boundary(hp, n, stencil, max_iter, solves=3):
    """The rate a caller of the reference's own interface sees (DESIGN.md 8,
    "The host boundary, measured"): HPCCG() through the C drop-in
    hpccg_hip_HPCCG (HPCCG.hpp:61-63) on a host HPC_Sparse_Matrix with host b
    and x -- device image cached by the first call, so each timed call is the
    PCIe copies of b and x plus the solve. Informational, never `value`. The
    drop-in prints the reference's residual lines (HPCCG.cpp:356, 372-373):
    stdout is pointed at stderr meanwhile, so the bench line stays the only
    stdout line."""
    import ctypes as C
    import numpy as np
    prob = hp.generate_matrix(n, n, n, use_7pt=stencil == 7)
    L = hp.lib()
    b = np.ascontiguousarray(prob.b)
    ni, nrm = C.c_int(0), C.c_double(0.0)
    times = np.zeros(7)
    walls, x = [], None
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        for i in range(solves + 1):
            x = prob.x
            t0 = time.perf_counter()
            rc = L.hpccg_hip_HPCCG(prob.A, b.ctypes.data, x.ctypes.data, max_iter, 0.0, C.byref(ni), C.byref(nrm),
                                   times.ctypes.data_as(C.POINTER(C.c_double)))
            hp._check(rc, "hpccg_hip_HPCCG")
            walls.append(time.perf_counter() - t0)
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)
    err = float(np.max(np.abs(x - 1.0)))
    prob.close()
    w = float(np.median(walls[1:]))
    return {"value": round(ni.value / w, 1), "unit": "CG iterations/s",
            "interface": "hpccg_hip_HPCCG (the reference's HPCCG() signature) on a host HPC_Sparse_Matrix, host b and x",
            "solves": solves, "median_wall_ms": round(w * 1e3, 3), "first_call_ms": round(walls[0] * 1e3, 1),
            "niters": ni.value, "x_minus_xexact_inf": err,
            "note": "PCIe copies of b and x included (device image cached by the first call, whose time includes "
                    "building it); informational, never value"}


def build_line(args, world, n, meas, roof, kernel, kfmt, fused, info, M_opts, rt, ranks, cpu, secondary,
               probe_report, trace_check=None, host_rate=None):
    """The one JSON line (pure: the CPU suite checks its schema for N > 1)."""
    it_per_s = meas["niters_total"] / meas["elapsed"]  # per rank: every rank runs the same iterations
    value = it_per_s * world
    nrow = info["nrow"]
    iter_bytes = 12.0 * info["nnz"] + 116.0 * nrow  # unfused reference sequence, SURVEY 8(d)
    step_s = meas["step_s"]
    es = meas["event_steps"]
    times_acc, niters_total = meas["times_acc"], meas["niters_total"]
    fupd = M_opts.get("fuse_update") == 1
    comm = ranks[0]["comm"]
    out = {
        "metric": f"CG iterations/sec + effective SpMV GB/s (% HBM peak), {args.stencil}-pt nx=ny=nz={n}",
        "value": round(value, 3),
        "unit": "CG iterations/s (per-GPU %d^3 slab iterations, summed over GPUs)" % n,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(meas["elapsed"] / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (generate_matrix stencil on the device; deterministic, no RNG)",
        "config": {
            "workload": f"HPCCG solve, {args.stencil}-pt {n}x{n}x{n} per GPU, z-stacked, "
                        f"max_iter={args.max_iter} ({args.max_iter - 1} CG iterations), tolerance 0",
            "nx": n, "ny": n, "nz_per_gpu": n, "stencil": args.stencil,
            "max_iter": args.max_iter,
            "parallelism": f"z-slab x{world}" + ("" if world == 1 else f" ({comm})"),
            "nnz_per_gpu": info["nnz"], "matrix_slots_per_gpu": info["slots"],
            "spmv_kernel": kernel, "matrix_format": FORMAT_NAMES[kfmt],
            "device_bytes_per_gpu": M_opts.get("device_bytes"),
            "graph_replay": bool(meas["graph_used"]),
            "placement_probe": probe_report,
            "options": {k: M_opts.get(k) for k in ("fuse_p", "fold", "x_defer", "x_ring", "graph_chunk", "nt", "a2_ring",
                                                   "nt_store", "fuse_update", "rhalo", "peer_allreduce", "halo_pull",
                                                   "resident_update")},
        },
        "cg_iterations_per_s_global": round(it_per_s, 3),
        "spmv_effective_gbs": roof["achieved"],
        "spmv_frac_hbm_peak": roof["frac"],
        "iteration_effective_gbs_credited": round(iter_bytes * it_per_s / 1e9, 1),
        "roofline": dict(roof, timing=meas["timing_src"]),
        # fused update: no update launch (its work is inside the SpMV launch above)
        "update_kernel_avg_us": round(meas["upd_ms"] / meas["upd_n"] * 1e3, 2) if (meas["upd_n"] and not fupd)
        else None,
        "check": {"x_minus_xexact_inf": meas["chk"][0], "final_normr_over_initial": meas["chk"][1],
                  "niters_per_solve": meas["it"], "resident_retries_max_over_ranks": meas["chk"][2]},
        # per-solve wall times on rank 0 (first/cold and median of the solves);
        # event steps launch eagerly with hipEvents and are slower than the graph replays
        "solve_ms": {"cold": round(meas["cold_s"] * 1e3, 3) if meas["cold_s"] is not None else None,
                     "median": round(sorted(step_s)[len(step_s) // 2] * 1e3, 3),
                     "min": round(min(step_s) * 1e3, 3), "max": round(max(step_s) * 1e3, 3),
                     "median_graph_replay": round(sorted(step_s[es:])[len(step_s[es:]) // 2] * 1e3, 3)
                     if len(step_s) > es else None},
        "times_per_step_s": {"total": times_acc[0] / args.steps, "ddot": times_acc[1] / args.steps,
                             "waxpby": times_acc[2] / args.steps, "sparsemv": times_acc[3] / args.steps,
                             "allreduce": times_acc[4] / args.steps, "halo": times_acc[5] / args.steps},
        # rank 0's device stamps (HPCCG.cpp:71-72 classes t4, t5) per CG iteration
        "per_iteration_us": {"allreduce": round(times_acc[4] / max(1, niters_total) * 1e6, 3),
                             "halo": round(times_acc[5] / max(1, niters_total) * 1e6, 3),
                             "total": round(meas["elapsed"] / max(1, niters_total) * 1e6, 3)},
        "runtime": dict(rt, comm=comm, ranks=ranks),
        "cpu_baseline": cpu,
    }
    if trace_check is not None:
        out["check"]["trace_vs_oracle"] = trace_check
    if host_rate is not None:
        out["host_boundary"] = host_rate
    if world > 1:
        out["multirank"] = multirank_summary(ranks, roof["bytes_per_launch"])
    if secondary is not None:
        out["secondary"] = secondary
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=200, help="nx = ny = nz per GPU")
    ap.add_argument("--stencil", type=int, default=27, choices=[27, 7])
    ap.add_argument("--max-iter", type=int, default=500)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-boundary", action="store_true",
                    help="N = 1: skip the host-interface rate (hpccg_hip_HPCCG with host b and x)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the other configs (N = 1: 27-pt 100^3, 7-pt 256^3; N > 1: 27-pt 100^3 per GPU)")
    ap.add_argument("--no-trace-check", action="store_true",
                    help="skip check.trace_vs_oracle (the oracle's rtrans trace of the global problem)")
    ap.add_argument("--trace-iters", type=int, default=60,
                    help="CG iterations of the oracle's trace the GPU trace is checked against (fewer if the "
                         "oracle's time budget is short)")
    ap.add_argument("--secondary-steps", type=int, default=10)
    ap.add_argument("--comm", default="auto", choices=["auto", "rccl", "host"],
                    help="N > 1: rccl (one rank per GPU), host (hpccg_hip_comm_init_host: ranks may share a GPU); "
                         "auto = rccl when there are at least N GPUs")
    ap.add_argument("--kernel", type=int, default=-1, help="SpMV kernel: 0 SELL-512, 1 A direct, 2 A pairs")
    ap.add_argument("--fuse-p", type=int, default=-1, help="p update inside the SpMV (-1 auto, 0 off)")
    ap.add_argument("--fold", type=int, default=-1, help="dot completion in the producer (-1 auto, 0 k_finalize)")
    ap.add_argument("--graph-chunk", type=int, default=-1, help="CG iterations per hipGraph (-1 default)")
    ap.add_argument("--x-defer", type=int, default=-1, help="batched x update (-1 default)")
    ap.add_argument("--x-ring", type=int, default=-1, help="x-update deferral depth = p ring length")
    ap.add_argument("--use-graph", type=int, default=-1, help="hipGraph replay (-1 default on)")
    ap.add_argument("--placement", type=int, default=0,
                    help="placement probe candidates at creation (default 0: off; -1 auto: 6 for images > 512 MB). "
                         "Off unless asked for: its gain depends on the box (DESIGN.md 4)")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VAL",
                    help="any other solver option (hpccg_hip_set_option), e.g. --set nt_store=0")
    ap.add_argument("--timeout", type=float, default=1200.0,
                    help="seconds before the run is abandoned (exit 124): the parent kills a relaunched job, "
                         "each rank's watchdog ends a run that outlives it (0: no limit)")
    ap.add_argument("--event-steps", type=int, default=1,
                    help="timed steps launched eagerly with hipEvents around every SpMV (the roofline's kernel "
                         "time); the other timed steps replay hipGraphs")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_distributed(args))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")

    stage = Stages(rank, args.timeout)
    stage("start", pid=os.getpid(), local_rank=local_rank, world=world)
    import torch
    import torch.distributed as dist
    hp = load_pkg()
    ndev = max(1, torch.cuda.device_count())
    comm = args.comm if args.comm != "auto" else ("rccl" if ndev >= world else "host")
    dev = local_rank % ndev
    torch.cuda.set_device(dev)
    hp.set_device(dev)
    if world > 1:
        init_gloo(dist, rank, world)
        if comm == "rccl":
            obj = [hp.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            hp.comm_init(obj[0], world, rank)
        else:
            hp.comm_init_host(world, rank)
    else:
        comm = "none"
    try:
        rt = hp.runtime_info()
    except AttributeError:  # an older library under A/B (HPCCG_HIP_LIB)
        rt = {"rccl_nranks": None, "pci_bus_id": None, "rccl_version": None, "rccl_rank": rank}
    stage("comm_init", comm=comm, device=dev, rccl_nranks=rt["rccl_nranks"], pci=rt["pci_bus_id"],
          rccl=rt["rccl_version"])

    n = args.n
    use_7pt = args.stencil == 7
    t0 = time.time()
    try:
        hp.set_placement_probe(args.placement)
    except AttributeError:  # an older library under A/B (HPCCG_HIP_LIB): no probe there
        pass
    M = hp.Matrix.generate(n, n, n, use_7pt=use_7pt)
    info = M.info()
    try:
        probe_us = M.placement()
        pick = M.get_option("placement_pick")
    except (AttributeError, hp.HPCCGError):
        probe_us, pick = [], 0
    for opt, val in (("spmv_kernel", args.kernel), ("fuse_p", args.fuse_p), ("fold", args.fold),
                     ("graph_chunk", args.graph_chunk), ("x_defer", args.x_defer), ("x_ring", args.x_ring),
                     ("use_graph", args.use_graph)):
        if val != -1:
            M.set_option(opt, val)
    for kv in args.set:
        key, _, val = kv.partition("=")
        M.set_option(key.strip(), int(val))
    stage("setup", seconds=f"{time.time() - t0:.2f}", nnz=info["nnz"], slots=info["slots"],
          kernel=M.get_option("spmv_kernel"), device_gb=f"{M.get_option('device_bytes') / 1e9:.2f}",
          transport={k: opt_or_none(M, k) for k in ("peer_allreduce", "halo_pull", "proto_auto_ok")})

    meas = measure(hp, torch, M, dev, args.max_iter, args.steps, args.warmup, args.event_steps, world, dist, stage)
    stage("timed", steps=args.steps, seconds=f"{meas['elapsed']:.3f}")
    roof, kernel, kfmt, fused, fupd = roofline_of(M, n, args.stencil, meas["spmv_avg_s"])
    M_opts = {k: opt_or_none(M, k) for k in ("fuse_p", "fold", "x_defer", "x_ring", "graph_chunk", "nt", "a2_ring",
                                             "nt_store", "fuse_update", "rhalo", "peer_allreduce", "halo_pull",
                                             "device_bytes", "resident_update")}
    ranks = gather_ranks(dist, world, rank_record(hp, M, rank, dev, comm, rt, meas))
    if world > 1:
        rt["pci_bus_ids"] = [r["pci_bus_id"] for r in ranks]
        rt["distinct_devices"] = len(set(rt["pci_bus_ids"]))
        if comm == "rccl" and (rt["rccl_nranks"] != world or rt["distinct_devices"] != world):
            log(f"[rank {rank}] WARNING: RCCL counts {rt['rccl_nranks']} ranks on {rt['distinct_devices']} distinct "
                f"devices for WORLD_SIZE={world}")
    else:
        rt["pci_bus_ids"] = [rt["pci_bus_id"]]
        rt["distinct_devices"] = 1
    M.close()

    host_rate = None
    if world == 1 and not args.no_host_boundary:
        try:
            stage("host_boundary_run")
            host_rate = host_boundary(hp, n, args.stencil, args.max_iter)
            stage("host_boundary", value=host_rate["value"])
        except Exception as e:  # reported, never silently dropped
            host_rate = {"error": repr(e)}

    secondary, sec_traces = None, {}
    if not args.no_secondary:
        secondary = []
        # N = 1: BASELINE.json's other single-GPU configs; N > 1: north_star's
        # second size, 100^3 per GPU, weak-scaled like the headline
        for n2, st2 in (((100, 27), (256, 7)) if world == 1 else ((100, 27),)):
            if (n2, st2) == (n, args.stencil):
                continue
            if world > 2 * ndev:
                # an emulation (--comm host, more than two ranks per GPU): the fused 100^3
                # launches of all the ranks sharing a GPU cannot be resident at once, and their
                # in-launch waits on each other's p.Ap would expire (creation refuses the matrix)
                secondary.append({"workload": f"{st2}-pt {n2}^3 per GPU", "skipped":
                                  f"{world} ranks share {ndev} GPU(s): the fused launches cannot all be resident"})
                continue
            try:
                stage("secondary_run", config=f"{st2}pt_{n2}")
                sec, tr2 = secondary_config(hp, torch, n2, st2, dev, args, world, dist, rank, comm, rt)
                secondary.append(sec)
                sec_traces[len(secondary) - 1] = (n2, st2, tr2)
                stage("secondary", config=f"{st2}pt_{n2}", value=sec["value"])
            except Exception as e:  # reported, never silently dropped
                secondary.append({"workload": f"{st2}-pt {n2}^3", "error": repr(e)})

    exit_code = 0
    if rank == 0:
        # rank 0's CPU work, after every GPU step, in a fresh child on the job's whole cpuset
        spec = {"traces": {}}
        if not args.no_cpu_baseline:
            spec["baseline"] = {"nx": n, "ny": n, "nz": n * world, "use_7pt": use_7pt, "world": world,
                                "budget_s": 15.0, "budget_1t_s": 10.0}
        if not args.no_trace_check:
            spec["traces"]["headline"] = {"nx": n, "ny": n, "nz": n * world, "use_7pt": use_7pt,
                                          "iters": args.trace_iters, "budget_s": 20.0}
            for i, (n2, st2, _) in sec_traces.items():
                spec["traces"][f"secondary{i}"] = {"nx": n2, "ny": n2, "nz": n2 * world, "use_7pt": st2 == 7,
                                                   "iters": args.trace_iters, "budget_s": 10.0}
        stage("cpu_child_run", baseline=bool(spec.get("baseline")), traces=len(spec["traces"]))
        child = run_cpu_child(spec, 900.0) if (spec.get("baseline") or spec["traces"]) else {}
        stage("cpu_child", seconds=child.get("seconds"), error=child.get("error"))
        cpu = None
        if not args.no_cpu_baseline:
            cpu = child.get("baseline") or {"error": child.get("error", "no baseline from the cpu child")}
        rtol = RTRANS_RTOL_1GPU if world == 1 else RTRANS_RTOL_MULTI
        ok_all = True

        def trace_record(name, gpu_tr, nx, nz_g, st):
            nonlocal ok_all
            ct = (child.get("traces") or {}).get(name)
            if ct is None or "error" in ct:
                return {"ok": None, "error": (ct or {}).get("error", child.get("error", "not run"))}
            rec = rtrans_check(gpu_tr, ct["trace"], rtol)
            rec.update({"oracle": f"oracle/hpccg_oracle.c HPCCG() on the global {nx}x{nx}x{nz_g} {st}-pt problem, "
                                  f"OpenMP {ct['threads']} threads, first {ct['iterations']} iterations "
                                  f"({ct['seconds']} s)",
                        "gpu": "rank 0's rtrans trace of the last timed solve (global, after the all-reduce)"})
            ok_all = ok_all and rec["ok"]
            return rec

        tchk = trace_record("headline", meas["trace"], n, n * world, args.stencil) if not args.no_trace_check \
            else None
        for i, (n2, st2, tr2) in sec_traces.items():
            if not args.no_trace_check:
                secondary[i]["check"]["trace_vs_oracle"] = trace_record(f"secondary{i}", tr2, n2, n2 * world, st2)
        out = build_line(args, world, n, meas, roof, kernel, kfmt, fused, info, M_opts, rt, ranks, cpu, secondary,
                         placement_report(args.placement, probe_us, pick), tchk, host_rate)
        retries = [meas["chk"][2]] + [s_["check"]["resident_retries_max_over_ranks"] for s_ in (secondary or [])
                                       if "check" in s_]
        if not ok_all:
            log("bench: the GPU trace does not match the oracle's within the stated tolerance; exiting 3")
            exit_code = 3
        elif any(retries):
            log(f"bench: resident launches were re-run after an expired wait ({retries}); exiting 3")
            exit_code = 3
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()  # rank 0's CPU leg runs while the others wait here
        hp.comm_destroy()
        dist.destroy_process_group()
    stage.done.set()
    return exit_code


if __name__ == "__main__":
    if len(sys.argv) == 4 and sys.argv[1] == "--cpu-child":
        cpu_child(sys.argv[2], sys.argv[3])
        sys.exit(0)
    sys.exit(main())
