"""Per-kernel durations and one stretch of the dispatch timeline from a
rocprofv3 --kernel-trace CSV (the in-process group's iteration).

    python tools/trace_timeline.py <kernel_trace.csv> [--anchor k_spmv_a] [--at 1000] [--count 22]
"""
import argparse
import collections
import csv
import re


def short(name):
    m = re.search(r"(k_\w+(<[^>]*>)?|__amd\w+|at::native::\w+)", name)
    return m.group(1) if m else name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--anchor", default="k_spmv_a<27, false, true")
    ap.add_argument("--at", type=int, default=1000, help="start at this occurrence of the anchor kernel")
    ap.add_argument("--count", type=int, default=22)
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    st = collections.defaultdict(list)
    for r in rows:
        st[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("kernel durations (us): launches, median, total")
    for k, v in st.items():
        v2 = sorted(v)
        print(f"  {k:52s} {len(v):6d} {v2[len(v2) // 2]:8.2f} {sum(v):11.1f}")
    idx = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]).startswith(args.anchor)]
    if len(idx) <= args.at:
        return
    i0 = idx[args.at]
    t0 = prev = int(rows[i0]["Start_Timestamp"])
    print(f"timeline from occurrence {args.at} of {args.anchor}: start (us), gap after the previous end, duration")
    for r in rows[i0:i0 + args.count]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        blocks = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        print(f"  {(s - t0) / 1e3:8.2f} gap={(s - prev) / 1e3:6.2f} dur={(e - s) / 1e3:7.2f} q={r['Queue_Id']} "
              f"blocks={blocks:5d} vgpr={r['VGPR_Count']:>3s} {short(r['Kernel_Name'])}")
        prev = e


if __name__ == "__main__":
    main()
