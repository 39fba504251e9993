"""Follow-up of tools/diag_carry.py: which disturbance changes a later solve.

    python tools/diag_carry2.py realloc      # pair kernel, one buffer moved at a time
    python tools/diag_carry2.py events N     # N rounds: event-timed eager solves on another b,
                                             # then a default solve and a fresh matrix, checked
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


def diff(a, b):
    if a[2].tobytes() == b[2].tobytes() and a[3].tobytes() == b[3].tobytes() and a[1] == b[1]:
        return "same"
    ta, tb = a[2], b[2]
    d = [i for i in range(min(len(ta), len(tb))) if ta[i] != tb[i]]
    return f"DIFF trace@{d[0] if d else -1} t0 {ta[0]:.10g}/{tb[0]:.10g} xdiff {np.max(np.abs(a[3] - b[3])):.3e}"


def realloc(prob):
    b = prob.b.copy()
    for kern in (PAIRS, DIRECT):
        for graph in (1, 0):
            for mode in (1, 0):
                for which in range(5):
                    M = hp.Matrix.from_hpc(prob)
                    M.set_option("spmv_kernel", kern)
                    M.set_option("use_graph", graph)
                    base = solve(M, b)
                    M.diag_realloc(which, mode)
                    print(f"k{kern} graph {graph} mode {mode} which {which}: {diff(base, solve(M, b))}", flush=True)
                    M.close()


def events(prob, rounds):
    b = prob.b.copy()
    b2 = np.full_like(b, 1.0000002384185791)
    t0 = float(np.sqrt(np.dot(b, b)))
    refs = {}
    for kern in (DIRECT, PAIRS):
        F = hp.Matrix.from_hpc(prob)
        F.set_option("spmv_kernel", kern)
        refs[kern] = (solve(F, b), solve(F, b2, 10))
        F.close()
    bad = 0
    for rep in range(rounds):
        for kern in (DIRECT, PAIRS):
            M = hp.Matrix.from_hpc(prob)
            M.set_option("spmv_kernel", kern)
            r1 = solve(M, b)
            M.set_option("event_timing", 1)
            ev = [solve(M, b2, 10) for _ in range(3)]
            M.set_option("event_timing", 0)
            r2 = solve(M, b)
            r3 = solve(M, b2, 10)
            out = [diff(refs[kern][0], r1), diff(refs[kern][1], ev[0]), diff(refs[kern][1], ev[2]),
                   diff(refs[kern][0], r2), diff(refs[kern][1], r3)]
            ok = all(o == "same" for o in out) and abs(r1[2][0] - t0) < 1e-9 * t0
            bad += not ok
            print(f"[{rep}] k{kern} {'ok' if ok else 'BAD'}: base {out[0]} | ev0 {out[1]} | ev2 {out[2]} | "
                  f"after {out[3]} | b2 {out[4]}", flush=True)
            M.close()
    print(f"DIAG_DONE bad={bad}", flush=True)


def main():
    hp.set_device(0)
    prob = hp.generate_matrix(40, 36, 30)
    if sys.argv[1] == "realloc":
        realloc(prob)
    else:
        events(prob, int(sys.argv[2]) if len(sys.argv) > 2 else 4)


if __name__ == "__main__":
    main()
