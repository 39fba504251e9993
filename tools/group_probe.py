"""Why does the two-member group's 100^3 SpMV take 56-58 us where one rank's
takes 40? Event-timed SpMV launch averages of the same unfused
launch (force_comm 1 on a 1-rank communicator) for: one matrix alone; the
same matrix with a second one allocated beside it; the second one; and the
two-member group (members alternate every launch).

    python tools/group_probe.py [--n 100]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import load_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--iters", type=int, default=100)
    args = ap.parse_args()
    import torch
    hp = load_pkg()
    hp.set_device(0)
    n = args.n
    hp.comm_init(hp.comm_unique_id(), 1, 0)

    def spmv_us(M, label):
        b, _, _ = M.vectors()
        x = torch.zeros(n ** 3, dtype=torch.float64, device="cuda:0")
        M.set_option("force_comm", 1)
        M.set_option("event_timing", 1)
        hp.HPCCG(M, b, x, max_iter=args.iters, device=True)
        kt = M.kernel_times()
        print(f"{label}: SpMV {kt['spmv_ms'] / kt['spmv_launches'] * 1e3:.1f} us, "
              f"update {kt['update_ms'] / kt['update_launches'] * 1e3:.1f} us", flush=True)

    M1 = hp.Matrix.generate(n, n, n)
    spmv_us(M1, "one matrix")
    spmv_us(M1, "one matrix again")
    M2 = hp.Matrix.generate(n, n, n)
    spmv_us(M1, "first, a second allocated")
    spmv_us(M2, "second")
    spmv_us(M1, "first again")
    M1.close()
    M2.close()
    hp.comm_destroy()
    # the group, eager with events is not available for groups: graph replay,
    # per-iteration time against the single-rank graph replay
    Ms = hp.group_generate(n, n, n, 2)
    xs = [torch.zeros(n ** 3, dtype=torch.float64, device="cuda:0") for _ in Ms]
    bs = [M.vectors()[0] for M in Ms]
    for _ in range(2):
        for x in xs:
            x.zero_()
        _, it, _, t = hp.group_HPCCG(Ms, bs, xs, max_iter=200)
        print(f"group of 2: {t[0] / it * 1e6:.1f} us per group iteration", flush=True)
    for M in Ms:
        M.close()


if __name__ == "__main__":
    main()
