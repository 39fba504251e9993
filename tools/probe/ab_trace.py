"""A/B: solve traces of two builds of libhpccg_hip.so (bitwise comparison of
the numerics after a kernel change that must not change any value)."""
import hashlib
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
lib = sys.argv[1]
spec = importlib.util.spec_from_file_location("hpccg_sycl_amd", os.path.join(ROOT, "hpccg-sycl_amd", "__init__.py"))
hp = importlib.util.module_from_spec(spec)
sys.modules["hpccg_sycl_amd"] = hp
spec.loader.exec_module(hp)
hp.LIB_PATH = lib
import torch  # noqa: E402
hp.set_device(0)
for dims, fold in [((20, 20, 20), 0), ((20, 20, 20), 1), ((64, 64, 48), 2), ((100, 100, 100), 0), ((100, 100, 100), 1)]:
    M = hp.Matrix.generate(*dims)
    M.set_option("fold", fold)
    b, _, _ = M.vectors()
    x = torch.zeros(dims[0] * dims[1] * dims[2], dtype=torch.float64, device="cuda:0")
    _, it, nr, _ = hp.HPCCG(M, b, x, max_iter=200, device=True)
    h = hashlib.sha256(M.last_trace().tobytes() + x.cpu().numpy().tobytes()).hexdigest()[:16]
    print(dims, fold, it, nr.hex(), h)
    M.close()
v = torch.arange(1, 100001, dtype=torch.float64, device="cuda:0").sin()
print("ddot", hp.ddot(100000, v, v).hex())
