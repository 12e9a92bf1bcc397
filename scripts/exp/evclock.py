"""Round 6: do HIP event durations agree with the host wall clock?
A ~1-s chain of GPU work timed by torch.cuda.Event (hipEventElapsedTime) and
by time.perf_counter around device syncs; also many short kernels (gaps)."""
import time

import torch

a = torch.randn(4096, 4096, device="cuda", dtype=torch.float32)
b = torch.randn(4096, 4096, device="cuda", dtype=torch.float32)
for _ in range(5):
    a @ b
torch.cuda.synchronize()
for label, reps, fn in (("matmul 4096^2 x", 400, lambda: a @ b), ("small add x", 20000, lambda: a.add_(1.0))):
    for trial in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        ev = e0.elapsed_time(e1)
        print(f"{label}{reps}: wall {wall:.2f} ms, events {ev:.2f} ms, wall/events {wall / ev:.4f}", flush=True)
