#!/usr/bin/env python3
"""Timeline of a rocprofv3 --kernel-trace (--memory-copy-trace) CSV run:
per-name count / average duration, and the idle gap before each operation
on the device, over the last operations in the trace.

usage: tools/trace_gaps.py <rocprofv3 output dir> [--last N]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def rows(d, pattern):
    out = []
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=120, help="operations listed from the end")
    ap.add_argument("--skip", type=int, default=0, help="drop this many operations at the end first")
    args = ap.parse_args()
    ops = []
    for r in rows(args.dir, "*kernel_trace.csv"):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:70]))
    for r in rows(args.dir, "*memory_copy_trace.csv"):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "")))
    ops.sort()
    stat = defaultdict(list)
    for s, e, n in ops:
        stat[n].append((e - s) / 1e3)
    for n, v in sorted(stat.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(v):6d} {sum(v) / len(v):10.2f} us  {n}")
    print("--- last ops: start offset, duration, gap before (us)")
    ops = ops[:len(ops) - args.skip]
    tail = ops[-args.last:]
    t0 = tail[0][0]
    prev_end = tail[0][0]
    for s, e, n in tail:
        print(f"{(s - t0) / 1e3:10.2f} {(e - s) / 1e3:9.2f} {(s - prev_end) / 1e3:9.2f}  {n}")
        prev_end = max(prev_end, e)


if __name__ == "__main__":
    main()
