"""Debug: the P=3 gather-plan group solve of tests/test_gpu_filemode.py, with
and without graph replay (prints progress; HPCCG_SEGV_TRACE=1 for a native
backtrace on a host crash)."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import torch  # noqa: E402

from conftest import load_pkg  # noqa: E402
import filemode  # noqa: E402

hp = load_pkg()
hp.set_device(0)
rp, cl, vl, x0, b, xe = filemode.general_system(600)
path = os.path.join(tempfile.mkdtemp(), "g.dat")
filemode.write(path, rp, cl, vl, x0, b, xe)
P = int(sys.argv[1]) if len(sys.argv) > 1 else 3
for graph in (0, 1):
    probs = [hp.read_HPC_row(path, r, P) for r in range(P)]
    parts = [(*p.to_csr(), p.start_row) for p in probs]
    Ms = hp.group_from_csr(parts, 600)
    print("created", [M.get_option("spmv_kernel") for M in Ms], [M.get_option("halo_mode") for M in Ms], flush=True)
    for M in Ms:
        M.set_option("use_graph", graph)
    xs = [torch.from_numpy(p.x).to("cuda:0") for p in probs]
    bs = [torch.from_numpy(p.b).to("cuda:0") for p in probs]
    _, it, nr, times = hp.group_HPCCG(Ms, bs, xs, max_iter=500)
    print("graph", graph, "it", it, "nr", nr, "used", Ms[0].get_option("graph_used"), flush=True)
