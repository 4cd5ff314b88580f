"""rocBLAS / hipBLASLt f64 GEMM rates at the policy MLP's shapes (reference point for the
hand-written f64 kernels: what the vendor library reaches on the same problem)."""
import torch

N = 190000
dev = torch.device("cuda:0")
cases = {"z2 = h1 W2^T [N,400]x[400,300]": (N, 400, 300),
         "dh1 = dz2 W2 [N,300]x[300,400]": (N, 300, 400),
         "square 8192^3": (8192, 8192, 8192)}
for name, (m, k, n) in cases.items():
    a = torch.randn(m, k, dtype=torch.float64, device=dev)
    b = torch.randn(k, n, dtype=torch.float64, device=dev)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 10 * 1e-3
    print(f"{name}: {t * 1e3:.3f} ms  {2.0 * m * n * k / t / 1e12:.1f} TF/s")
# dW2 = dz2^T h1 (reduction over N): the transposed-A form
a = torch.randn(N, 300, dtype=torch.float64, device=dev)
b = torch.randn(N, 400, dtype=torch.float64, device=dev)
for _ in range(3):
    c = a.t() @ b
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    c = a.t() @ b
e1.record()
torch.cuda.synchronize()
t = e0.elapsed_time(e1) / 10 * 1e-3
print(f"dW2 = dz2^T h1 [300,N]x[N,400]: {t * 1e3:.3f} ms  {2.0 * N * 300 * 400 / t / 1e12:.1f} TF/s")
