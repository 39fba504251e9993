"""Split the SpMV dispatches of a tools/placement_pmc.py run under
rocprofv3 --pmc into phase A (first half) and phase B (second half) and print
each counter's mean per dispatch per phase and the B/A ratio.

    python tools/pmc_phases.py gpurun_out/pmcpl/p*/run_counter_collection.csv
"""
import csv
import sys
from collections import defaultdict


def main():
    for path in sys.argv[1:]:
        per = defaultdict(dict)  # dispatch -> counter -> value
        order = []
        with open(path) as f:
            for row in csv.DictReader(f):
                if "k_spmv_a2r" not in row["Kernel_Name"]:
                    continue
                d = int(row["Dispatch_Id"])
                if d not in per:
                    order.append(d)
                per[d][row["Counter_Name"]] = float(row["Counter_Value"])
        order.sort()
        half = len(order) // 2
        ph = {"A": order[:half], "B": order[half:]}
        names = sorted({c for d in order for c in per[d]})
        print(f"== {path}: {len(order)} SpMV dispatches")
        for c in names:
            m = {k: sum(per[d][c] for d in v) / max(1, len(v)) for k, v in ph.items()}
            ratio = m["B"] / m["A"] if m["A"] else float("nan")
            print(f"  {c:48s} A {m['A']:16.1f}  B {m['B']:16.1f}  B/A {ratio:7.3f}")


if __name__ == "__main__":
    main()
