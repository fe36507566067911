"""Ceiling probe: rocBLAS f64 GEMMs (torch.matmul) at the chain-batched shapes of SURVEY §8d
(C chains: X·W = [B×D]·[D×10C], Xᵀ·diff = [D×B]·[B×10C]).  Usage: python tools/probe_dgemm.py [C]"""
import sys
import time

import torch

C = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
B, D, K = 500, 784, 10
dev = torch.device("cuda", 0)
X = torch.rand(B, D, dtype=torch.float64, device=dev)
W = torch.rand(D, K * C, dtype=torch.float64, device=dev)
G = torch.rand(B, K * C, dtype=torch.float64, device=dev)
for name, f in (("X.W", lambda: X @ W), ("Xt.diff", lambda: X.t() @ G)):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    n = 20
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    print("%-8s C=%d  %.1f us  %.1f TFLOP/s (%.1f %% of 78.6)" % (name, C, dt * 1e6, 2 * B * D * K * C / dt / 1e12,
                                                           2 * B * D * K * C / dt / 1e12 / 78.6 * 100))
