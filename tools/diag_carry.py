"""State carried between solves: run sequences that
solve one matrix, disturb it (placement probe, eager event-timed solves with
another b, buffer moves), solve again, and report where the second solve
departs from the first (first differing trace index, initial residual, pick).

    python tools/diag_carry.py [reps]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

hp = ge._import_pkg()
DIRECT, PAIRS = 1, 2


def solve(M, b, it=40):
    x = np.zeros(len(b))
    _, n, nr, _ = hp.HPCCG(M, b, x, max_iter=it)
    return n, nr, M.last_trace().copy(), x


def cmp(tag, a, b, extra=""):
    same = a[0] == b[0] and a[1] == b[1] and a[2].tobytes() == b[2].tobytes() and a[3].tobytes() == b[3].tobytes()
    if same:
        print(f"{tag}: same {extra}", flush=True)
        return True
    ta, tb = a[2], b[2]
    m = min(len(ta), len(tb))
    d = [i for i in range(m) if ta[i] != tb[i]]
    first = d[0] if d else -1
    print(f"{tag}: DIFF first trace index {first} t0 {ta[0]!r} vs {tb[0]!r} normr {a[1]!r} vs {b[1]!r} "
          f"x0 maxdiff {np.max(np.abs(a[3] - b[3])):.3e} {extra}", flush=True)
    if first >= 0:
        lo = max(0, first - 1)
        print("   base ", ta[lo:first + 3], "\n   after", tb[lo:first + 3], flush=True)
    return False


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    hp.set_device(0)
    prob = hp.generate_matrix(40, 36, 30)
    b = prob.b.copy()
    b2 = np.full_like(b, 1.0000002384185791)
    bad = 0
    for rep in range(reps):
        for kern in (DIRECT, PAIRS):
            # A: placement probe
            M = hp.Matrix.from_hpc(prob)
            M.set_option("spmv_kernel", kern)
            base = solve(M, b)
            us = M.probe_placement(3)
            pick = M.get_option("placement_pick")
            bad += not cmp(f"[{rep}] k{kern} probe", base, solve(M, b), f"pick {pick:#x} us {np.round(us, 1)}")
            M.close()
            # B: eager event-timed solves on another b, no buffer moved
            M = hp.Matrix.from_hpc(prob)
            M.set_option("spmv_kernel", kern)
            base = solve(M, b)
            M.set_option("event_timing", 1)
            for _ in range(3):
                solve(M, b2, 10)
            M.set_option("event_timing", 0)
            bad += not cmp(f"[{rep}] k{kern} eager-b2", base, solve(M, b))
            # B2: the b2 solve against a fresh matrix's b2 solve
            F = hp.Matrix.from_hpc(prob)
            F.set_option("spmv_kernel", kern)
            bad += not cmp(f"[{rep}] k{kern} b2-vs-fresh", solve(F, b2), solve(M, b2))
            F.close()
            M.close()
            # C: buffers moved, no other solve
            M = hp.Matrix.from_hpc(prob)
            M.set_option("spmv_kernel", kern)
            base = solve(M, b)
            for which in range(4):
                M.diag_realloc(which, int(os.environ.get("DIAG_REALLOC_MODE", "1")))
            bad += not cmp(f"[{rep}] k{kern} realloc", base, solve(M, b))
            M.close()
    print(f"DIAG_DONE bad={bad}", flush=True)


if __name__ == "__main__":
    main()
