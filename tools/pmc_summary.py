#!/usr/bin/env python3
"""Turn a tools/gpu_profile.sh run into committed evidence under profiles/.

* kernel stats of the bench command (rocprofv3 --kernel-trace --stats)
* HBM traffic per SpMV launch from two separate --pmc passes (FETCH_SIZE,
  WRITE_SIZE; KiB units). gfx950 correction (MI355X_MICROARCH.md, HBM):
  FETCH_SIZE reports 1/2 of a wide coalesced stream; the factor is
  calibrated here on k_stream_a, which reads exactly 8 * a_slots bytes (the
  SELL-512-A values, 16 B non-temporal loads per lane: the SpMV's own matrix
  access pattern) and writes 8 * nrow.

usage: tools/pmc_summary.py <prof_dir> <tag> <nx> [<bench_json_log>] [<stencil 27|7>]
"""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


FORMATS = {
    "k_spmv_sell": "SELL-512 (8 B value + int32 column per slot)",
    "k_spmv_a": "SELL-512-A (8 B value per offset-aligned slot, holes 0.0), x read at the slice's offsets",
    "k_spmv_a2": "SELL-512-A (8 B value per offset-aligned slot, holes 0.0), x from LDS windows shared by slice pairs",
    "k_spmv_a2r": "SELL-512-A (8 B value per offset-aligned slot, holes 0.0), x from LDS windows shared by slice pairs, "
                  "values streamed HBM -> LDS by per-wave LDS-DMA rings",
    "k_cg_persist": "SELL-512-A (8 B value per offset-aligned slot, holes 0.0), x read at the slice's offsets, one "
                    "block per slice pair resident for the whole solve: one launch runs every iteration",
    "k_spmv_ar": "SELL-512-A (8 B value per offset-aligned slot, holes 0.0), x read at the slice's offsets, one block "
                 "per slice pair, every block resident: the update applied from registers (no Ap stream)",
}


def newest(pattern):
    """The most recent file matching pattern (gpurun_out keeps older runs)."""
    files = glob.glob(pattern)
    if not files:
        raise FileNotFoundError(pattern)
    return max(files, key=os.path.getmtime)


def counters(path):
    agg = defaultdict(list)
    for row in csv.DictReader(open(path)):
        agg[(row["Kernel_Name"], row["Counter_Name"])].append(float(row["Counter_Value"]))
    return agg


def pick(agg, needle, counter):
    """Average over dispatches of the most-dispatched kernel matching needle
    (a substring or a tuple of substrings; the in-loop SpMV, not the prologue one)."""
    needles = needle if isinstance(needle, tuple) else (needle,)
    best = None
    for (k, c), v in agg.items():
        if any(nd in k for nd in needles) and c == counter and (best is None or len(v) > len(best[1])):
            best = (k, v)
    if best is None:
        raise KeyError(needle)
    return sum(best[1]) / len(best[1]), best[0]


def main():
    prof, tag, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    bench_log = sys.argv[4] if len(sys.argv) > 4 else None
    outdir = os.path.join(ROOT, "profiles", tag)
    os.makedirs(outdir, exist_ok=True)
    stats = newest(os.path.join(prof, "stats", "*", "*_kernel_stats.csv"))
    shutil.copy(stats, os.path.join(outdir, "kernel_stats.csv"))
    dom = glob.glob(os.path.join(prof, "stats", "*", "*_domain_stats.csv"))
    if dom:
        shutil.copy(newest(os.path.join(prof, "stats", "*", "*_domain_stats.csv")),
                    os.path.join(outdir, "domain_stats.csv"))
    fetch = counters(newest(os.path.join(prof, "fetch", "*", "*_counter_collection.csv")))
    write = counters(newest(os.path.join(prof, "write", "*", "*_counter_collection.csv")))
    for src, name in [("fetch", "pmc_fetch_size.csv"), ("write", "pmc_write_size.csv")]:
        shutil.copy(newest(os.path.join(prof, src, "*", "*_counter_collection.csv")),
                    os.path.join(outdir, name))

    stencil = int(sys.argv[5]) if len(sys.argv) > 5 else 27
    nrow = n ** 3
    # the uniform SELL-512-A image of the stencil problem
    width = 27 if stencil == 27 else 7
    slots = ((nrow + 511) // 512) * 512 * width
    nnz = (3 * n - 2) ** 3 if stencil == 27 else 7 * n ** 3 - 6 * n * n
    stream_read = 8.0 * slots  # k_stream_a reads the 8 B/slot A image
    f_stream, _ = pick(fetch, "k_stream_a", "FETCH_SIZE")
    w_stream, _ = pick(write, "k_stream_a", "WRITE_SIZE")
    fetch_factor = stream_read / (f_stream * 1024.0)
    SPMV = ("k_spmv_sell<", "k_spmv_a<", "k_spmv_a2<", "k_spmv_a2r<", "k_spmv_ar<")
    # (the persistent launch, when the solve ran one: its single dispatch, not the prologue's SpMV)
    if any("k_cg_persist<" in k for k, _ in fetch):
        SPMV = ("k_cg_persist<",)
    f_spmv, kname = pick(fetch, SPMV, "FETCH_SIZE")
    w_spmv, _ = pick(write, SPMV, "WRITE_SIZE")
    # the persistent launch (k_cg_persist) runs every iteration of a solve in
    # one dispatch: its counters and its duration are divided by the
    # iterations of that dispatch (pmc_workload: --iters - 1; the bench:
    # max_iter - 1), so every figure below is per iteration
    persist = "k_cg_persist<" in kname
    pmc_iters = int(os.environ.get("PMC_ITERS", "32")) - 1 if persist else 1
    spmv_read = f_spmv * 1024.0 * fetch_factor / pmc_iters
    spmv_write = w_spmv * 1024.0 / pmc_iters
    targs = re.search(r"(?:k_spmv\w*|k_cg_persist)<([^>]*)>", kname).group(1).split(",")
    # k_spmv_a<kW, kNT, kFuse, kPre>, k_spmv_a2<kNT, kFuse, kPre>, k_spmv_a2r<kFuse, kW, kR>,
    # k_spmv_sell<kNT> (never fused)
    if "k_spmv_a<" in kname:
        fuse_p = targs[2].strip() == "true"
    elif "k_spmv_a2r<" in kname:
        fuse_p = targs[0].strip() == "true"
    elif "k_spmv_a2<" in kname:
        fuse_p = targs[1].strip() == "true"
    elif "k_spmv_ar<" in kname or persist:  # always fused (p and the update)
        fuse_p = True
    else:
        fuse_p = False
    algo = 12.0 * nnz + 20.0 * nrow + 16.0 * nrow + (24.0 * nrow if fuse_p else 0.0)
    # the bytes the format must move: 8 B per stored slot, + r, p_{k-1} read and
    # p_k, Ap written (fused) or p read and Ap written
    compulsory = 8.0 * slots + (32.0 if fuse_p else 16.0) * nrow
    # x_defer 2: trailing blocks of every launch but the first iteration's
    # apply the deferred x terms of 1/q of the rows (x read and written, q p's)
    bench = None
    if bench_log and os.path.exists(bench_log):
        lines = [l for l in open(bench_log) if l.startswith("{")]
        bench = json.loads(lines[-1]) if lines else None
    opts = bench["config"]["options"] if bench else {}
    side = 0.0
    if opts.get("x_defer") == 2 and not persist:  # (persistent: x in registers)
        q = opts["x_ring"] - 1
        launches = len(fetch[(kname, "FETCH_SIZE")])
        side = (16.0 + 8.0 * q) / q * nrow * (launches - 1) / launches
        compulsory += side
    resident = "k_spmv_ar<" in kname or persist
    # fused update blocks: r, Ap read; r written (resident: applied from registers, r written
    # instead of Ap -- the same 32 B per row as above, nothing more)
    upd = 24.0 * nrow if (opts.get("fuse_update") == 1 and not resident) else 0.0
    compulsory += upd

    avg_ns = None
    calls = -1
    # the kernel the PMC passes measured (the stats run may also hold other
    # SpMV kernels, e.g. the prologue's unfused launch)
    for row in csv.DictReader(open(stats)):
        if row["Name"] == kname and int(row["Calls"]) > calls:
            avg_ns, calls = float(row["AverageNs"]), int(row["Calls"])
    if persist and avg_ns:
        bench_iters = (bench["config"].get("max_iter", 500) - 1) if bench else 499
        avg_ns /= bench_iters
    out = {
        "tag": tag,
        "problem": f"{stencil}-pt {n}^3, SELL-512 width {width} ({slots} slots, nnz {nnz}); "
                   + FORMATS.get(re.search(r"(k_spmv\w*|k_cg_persist)<", kname).group(1), kname),
        "kernel": kname,
        "fuse_p": fuse_p,
        "bytes_formula": "12 nnz + 20 n + 16 n" + (" + 24 n" if fuse_p else ""),
        "format_compulsory_bytes_per_launch": compulsory,
        "x_defer": opts.get("x_defer"),
        "side_flush_bytes_per_launch": side,
        "fuse_update": opts.get("fuse_update", 0),
        "fused_update_bytes_per_launch": upd,
        "resident_update": opts.get("resident_update", 1 if resident else 0) if resident else 0,
        "per_iteration_of_one_dispatch": persist,
        "fetch_size_kib_raw": f_spmv,
        "write_size_kib_raw": w_spmv,
        "fetch_calibration": {"kernel": "k_stream_a", "known_read_bytes": stream_read,
                              "fetch_size_kib": f_stream, "factor": round(fetch_factor, 4),
                              "write_size_kib": w_stream, "known_write_bytes": 8.0 * nrow},
        "spmv_hbm_read_bytes_per_launch": spmv_read,
        "spmv_hbm_write_bytes_per_launch": spmv_write,
        "spmv_hbm_bytes_per_launch": spmv_read + spmv_write,
        "spmv_algorithmic_bytes_per_launch": algo,
        "traffic_over_algorithmic": (spmv_read + spmv_write) / algo,
        "traffic_over_compulsory": (spmv_read + spmv_write) / compulsory,
        "rocprof_avg_spmv_ns": avg_ns,
        "rocprof_spmv_traffic_GBs": (spmv_read + spmv_write) / avg_ns if avg_ns else None,
        "rocprof_spmv_compulsory_GBs": compulsory / avg_ns if avg_ns else None,
        "rocprof_spmv_credited_GBs": algo / avg_ns if avg_ns else None,
    }
    # every kernel of the pmc workload: corrected HBM bytes per launch
    per_kernel = {}
    for (k, c), v in fetch.items():
        if c != "FETCH_SIZE":
            continue
        short = re.sub(r"^void |hpccg::\(anonymous namespace\)::|\(.*$", "", k)
        wv = write.get((k, "WRITE_SIZE"), [0.0])
        per_kernel[short] = {"launches": len(v),
                             "read_bytes": round(sum(v) / len(v) * 1024.0 * fetch_factor),
                             "write_bytes": round(sum(wv) / len(wv) * 1024.0)}
    out["per_kernel_hbm_bytes_per_launch"] = per_kernel
    if bench:
        out["bench_avg_launch_us"] = bench["roofline"]["avg_launch_us"]
        out["bench_value"] = bench["value"]
        shutil.copy(bench_log, os.path.join(outdir, "bench_line.json"))  # as printed
        # the same line with roofline.traffic from THIS run's PMC passes (bench.py
        # reads the committed profiles/pmc_*.json, which predate this run)
        ann = json.loads(json.dumps(bench))
        rl = ann["roofline"]
        t = spmv_read + spmv_write
        rl["traffic"] = t
        rl["traffic_source"] = (f"profiles/{tag}/summary.json: rocprofv3 FETCH_SIZE (x{fetch_factor:.4f}, calibrated on "
                                f"k_stream_a) + WRITE_SIZE passes of this evidence run (separate processes)")
        rl["traffic_gbs"] = round(t / (rl["avg_launch_us"] * 1e3), 1)
        rl["traffic_frac"] = round(rl["traffic_gbs"] / rl["peak"], 4)
        with open(os.path.join(outdir, "bench_line_with_traffic.json"), "w") as f:
            json.dump(ann, f)
    with open(os.path.join(ROOT, "profiles", f"pmc_spmv_{stencil}pt_{n}.json"), "w") as f:
        json.dump(out, f, indent=1)
    with open(os.path.join(outdir, "summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
