"""fp64 GEMM rate of the vendor library (torch.matmul -> hipBLASLt/rocBLAS) on
MI355X: the attainable v_mfma_f64 rate to compare k_gp_var against."""
import json
import torch

res = {}
for n in (4096, 8192):
    a = torch.randn(n, n, dtype=torch.float64, device="cuda")
    b = torch.randn(n, n, dtype=torch.float64, device="cuda")
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    e0.record()
    for _ in range(reps):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    res[n] = {"ms": ms, "tflops": 2 * n ** 3 / ms / 1e9, "frac_of_78.6": 2 * n ** 3 / ms / 1e9 / 78.6}
print(json.dumps(res))
