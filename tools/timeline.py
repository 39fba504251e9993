#!/usr/bin/env python3
"""Block timeline of the SpMV launch: the ring pair kernel (k_spmv_a2r<true,
27, 3>, 200^3) -- where a block's life goes (state read, window staging, slot
loop, epilogue + dot hand-off), how the blocks overlap on each CU, the
launch's head and tail -- or the direct kernel with the fused update (100^3,
7-pt 256^3): unit, side-flush and update blocks, the update blocks' wait for
the p.Ap total, residency per role. Diagnostics only (option dbg_timeline,
hpccg_hip_diag_timeline).

usage: tools/timeline.py [--n 200] [--stencil 27] [--iters 40] [--json out.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import load_pkg  # noqa: E402

TICK_US = 0.01  # s_memrealtime: 100 MHz


def pct(v, q):
    return float(np.percentile(v, q))


def analyse(tl):
    blk = (tl[:, 0] & 0xFFFFFFFF).astype(np.int64)
    hwid = (tl[:, 0] >> 32).astype(np.int64)
    t = tl[:, 1:6].astype(np.int64)
    xcc = tl[:, 6].astype(np.int64)
    ks = tl[:, 7].astype(np.int64)
    ok = t[:, 0] > 0
    blk, hwid, t, xcc, ks = blk[ok], hwid[ok], t[ok], xcc[ok], ks[ok]
    t0 = t[:, 0].min()
    t = (t - t0) * TICK_US  # us from the first block's entry
    span = t[:, 4].max()
    ph = {"state": t[:, 1] - t[:, 0], "staging": t[:, 2] - t[:, 1], "slots": t[:, 3] - t[:, 2],
          "epilogue": t[:, 4] - t[:, 3], "life": t[:, 4] - t[:, 0]}
    out = {"units": int(len(t)), "iterations_seen": sorted(set(int(k) for k in ks))[:4],
           "span_us": round(float(span), 2),
           "phases_us": {k: {"mean": round(float(v.mean()), 3), "p10": round(pct(v, 10), 3),
                             "p50": round(pct(v, 50), 3), "p90": round(pct(v, 90), 3),
                             "max": round(float(v.max()), 3)} for k, v in ph.items()},
           "phase_share_of_life": {k: round(float(ph[k].sum() / ph["life"].sum()), 4)
                                   for k in ("state", "staging", "slots", "epilogue")}}
    # head: until every CU slot is busy; tail: after the last block started
    starts = np.sort(t[:, 0])
    ends = np.sort(t[:, 4])
    out["head_us_first_512_entries"] = round(float(starts[min(511, len(starts) - 1)]), 2)
    out["tail_us_after_last_entry"] = round(float(span - starts[-1]), 2)
    out["tail_us_after_p99_end"] = round(float(span - ends[int(0.99 * len(ends))]), 2)
    # per CU: (xcc, se, sh, cu) from HW_ID (cu_id [11:8], sh_id [12], se_id [15:13])
    cu = xcc * 4096 + ((hwid >> 8) & 0xFF)
    cus = np.unique(cu)
    out["cus_seen"] = int(len(cus))
    # concurrency: on each CU, time-weighted number of resident blocks, and of
    # blocks in the slot loop (the value stream)
    res_w, str_w, gap = [], [], []
    grid = np.linspace(0, span, 2000)
    busy_all = np.zeros_like(grid)
    stream_all = np.zeros_like(grid)
    for c in cus:
        m = cu == c
        tc = t[m]
        res = ((grid[:, None] >= tc[None, :, 0]) & (grid[:, None] < tc[None, :, 4])).sum(1)
        stm = ((grid[:, None] >= tc[None, :, 2]) & (grid[:, None] < tc[None, :, 3])).sum(1)
        busy_all += res
        stream_all += stm
        res_w.append(res.mean())
        str_w.append(stm.mean())
        # dispatch gap: a block's end to the next entry on the same CU
        e = np.sort(tc[:, 4])
        s = np.sort(tc[:, 0])
        for x in e:
            nxt = s[s >= x]
            if len(nxt):
                gap.append(nxt[0] - x)
    out["per_cu_mean_resident_blocks"] = round(float(np.mean(res_w)), 3)
    out["per_cu_mean_streaming_blocks"] = round(float(np.mean(str_w)), 3)
    if gap:
        g = np.array(gap)
        out["dispatch_gap_us"] = {"mean": round(float(g.mean()), 3), "p50": round(pct(g, 50), 3),
                                  "p90": round(pct(g, 90), 3)}
    # the chip in 10 slices of the span: resident and streaming blocks per CU
    n = len(cus)
    prof = []
    for i in range(10):
        sl = slice(i * 200, (i + 1) * 200)
        prof.append([round(float(busy_all[sl].mean() / n), 2), round(float(stream_all[sl].mean() / n), 2)])
    out["span_deciles_resident_streaming_per_cu"] = prof
    return out


ROLES = {0: "unit", 1: "side", 2: "ghost", 3: "update"}


def analyse_direct(tl):
    """Rows of the direct kernel's timeline (one per block): block | HW_ID <<
    32, entry, state read / p.Ap ready, slot loop done, end, role, XCC."""
    t = tl[:, 1:5].astype(np.int64)
    role = tl[:, 5].astype(np.int64)
    ok = (t[:, 0] > 0) & (t[:, 3] >= t[:, 0])
    t, role, hw, xcc = t[ok], role[ok], (tl[ok, 0] >> 32).astype(np.int64), tl[ok, 6].astype(np.int64)
    t0 = t[:, 0].min()
    t = (t - t0) * TICK_US
    t[t < 0] = np.nan  # unset stamps (0) of roles that skip a phase
    span = float(np.nanmax(t[:, 3]))
    out = {"blocks": int(len(t)), "span_us": round(span, 2), "roles": {}}
    for r, name in ROLES.items():
        m = role == r
        if not m.any():
            continue
        tr = t[m]
        d = {"blocks": int(m.sum()),
             "first_entry_us": round(float(np.nanmin(tr[:, 0])), 2),
             "last_end_us": round(float(np.nanmax(tr[:, 3])), 2),
             "life_us": {"mean": round(float(np.nanmean(tr[:, 3] - tr[:, 0])), 3),
                         "p50": round(float(np.nanpercentile(tr[:, 3] - tr[:, 0], 50)), 3),
                         "p90": round(float(np.nanpercentile(tr[:, 3] - tr[:, 0], 90)), 3)}}
        if r == 0:
            d["state_us_mean"] = round(float(np.nanmean(tr[:, 1] - tr[:, 0])), 3)
            d["slots_us_mean"] = round(float(np.nanmean(tr[:, 2] - tr[:, 1])), 3)
            d["epilogue_us_mean"] = round(float(np.nanmean(tr[:, 3] - tr[:, 2])), 3)
        if r == 3:
            d["wait_us_mean"] = round(float(np.nanmean(tr[:, 1] - tr[:, 0])), 3)
            d["wait_us_p90"] = round(float(np.nanpercentile(tr[:, 1] - tr[:, 0], 90)), 3)
            d["work_us_mean"] = round(float(np.nanmean(tr[:, 3] - tr[:, 1])), 3)
            d["first_ready_us"] = round(float(np.nanmin(tr[:, 1])), 2)
        out["roles"][name] = d
    # per CU residency over the span, by role
    cu = xcc * 4096 + ((hw >> 8) & 0xFF)
    cus = np.unique(cu)
    grid = np.linspace(0, span, 1000)
    prof = {}
    for r, name in ROLES.items():
        m = role == r
        if not m.any():
            continue
        res = ((grid[:, None] >= t[m][None, :, 0]) & (grid[:, None] < t[m][None, :, 3])).sum(1) / len(cus)
        prof[name] = [round(float(res[i * 100:(i + 1) * 100].mean()), 2) for i in range(10)]
    out["cus_seen"] = int(len(cus))
    out["span_deciles_resident_per_cu"] = prof
    gap = []
    for c in cus:
        mc = cu == c
        e = np.sort(t[mc, 3])
        st = np.sort(t[mc, 0])
        idx = np.searchsorted(st, e)
        nxt = idx < len(st)
        gap.extend((st[idx[nxt]] - e[nxt]).tolist())
    if gap:
        g = np.array(gap)
        out["dispatch_gap_us"] = {"mean": round(float(g.mean()), 3), "p50": round(float(np.percentile(g, 50)), 3)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--stencil", type=int, default=27, choices=[27, 7])
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--json", default=None)
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VAL")
    args = ap.parse_args()
    import torch
    hp = load_pkg()
    hp.set_device(0)
    M = hp.Matrix.generate(args.n, args.n, args.n, use_7pt=args.stencil == 7)
    direct = M.get_option("spmv_kernel") == 1
    for kv in args.set:
        k, _, v = kv.partition("=")
        M.set_option(k.strip(), int(v))
    b = M.vectors()[0]
    x = torch.zeros(args.n ** 3, dtype=torch.float64, device="cuda:0")
    res = {}
    for mode in (("eager",) if direct else ("graph", "eager")):  # direct: no-op launches would half-write rows
        M.set_option("use_graph", 1 if mode == "graph" else 0)
        M.set_option("dbg_timeline", 1)
        x.zero_()
        hp.HPCCG(M, b, x, max_iter=args.iters, device=True)  # warm (capture)
        x.zero_()
        hp.HPCCG(M, b, x, max_iter=args.iters, device=True)
        tl = M.diag_timeline()
        res[mode] = analyse_direct(tl) if direct else analyse(tl)
        M.set_option("dbg_timeline", 0)
    print(json.dumps(res, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)
    M.close()


if __name__ == "__main__":
    main()
