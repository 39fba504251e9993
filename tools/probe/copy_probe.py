import time, torch, numpy as np, os
n = 8_000_000
def t(f, reps=5):
    f(); torch.cuda.synchronize()
    ts=[]
    for _ in range(reps):
        t0=time.perf_counter(); f(); torch.cuda.synchronize(); ts.append(time.perf_counter()-t0)
    return min(ts)*1e3
a = np.random.rand(n); d = torch.empty(n, dtype=torch.float64, device="cuda")
pa = torch.from_numpy(a)
pin = torch.empty(n, dtype=torch.float64).pin_memory()
print("cpus", len(os.sched_getaffinity(0)))
print("H2D pageable ms", t(lambda: d.copy_(pa)))
print("H2D pinned ms", t(lambda: d.copy_(pin, non_blocking=True)))
print("D2H pageable ms", t(lambda: pa.copy_(d)))
print("D2H pinned ms", t(lambda: pin.copy_(d, non_blocking=True)))
b = np.empty_like(a)
print("memcpy 1 thread ms", t(lambda: np.copyto(b, a)))
print("memcpy to pinned ms", t(lambda: pin.numpy().__setitem__(slice(None), a)))
