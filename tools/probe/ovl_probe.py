import sys, time, os
sys.path.insert(0, os.getcwd())
from bench import load_pkg
import torch
hp = load_pkg(); hp.set_device(0)
Ms = hp.group_generate(100, 100, 100, 2)
bs = [M.vectors()[0] for M in Ms]
xs = [torch.zeros(100**3, dtype=torch.float64, device="cuda:0") for _ in Ms]
for ovl, mi in ((0, 500), (1, 500), (1, 497), (0, 497), (1, 500)):
    for M in Ms:
        M.set_option("use_graph", 1); M.set_option("overlap", ovl)
    ts = []
    for rep in range(4):
        for x in xs: x.zero_()
        torch.cuda.synchronize(); t0 = time.perf_counter()
        it = hp.group_HPCCG(Ms, bs, xs, max_iter=mi)[1]
        torch.cuda.synchronize(); ts.append((time.perf_counter() - t0) * 1e3)
    print("ovl", ovl, "max_iter", mi, "iters", it, "graph_used", Ms[0].get_option("graph_used"), "ms", [round(t, 1) for t in ts], flush=True)
