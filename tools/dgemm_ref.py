"""Library comparison point for the GRM kernel: torch fp64 GEMM (rocBLAS/hipBLASLt) computing the
same G = Zᵀ Z (full square, n x n, K = p) and torch's SYRK-shaped alternative. Prints TF/s both
as library flops (2 n² p) and as the GRM's algorithmic flops (n (n+1) p)."""
import sys
import time

import torch

n, p = (int(a) for a in sys.argv[1:3]) if len(sys.argv) > 2 else (5000, 50000)
Z = torch.randn(p, n, dtype=torch.float64, device="cuda")
for _ in range(2):
    G = Z.T @ Z
torch.cuda.synchronize()
reps = 5
t0 = time.perf_counter()
for _ in range(reps):
    G = Z.T @ Z
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / reps
print(f"torch fp64 Z^T Z n={n} p={p}: {dt*1e3:.2f} ms  library {2*n*n*p/dt/1e12:.1f} TF/s  "
      f"algorithmic(triangle) {n*(n+1)*p/dt/1e12:.1f} TF/s")
