"""Timing probe: C independent SGHMC chains sharing each minibatch on one GPU (kernel-per-phase
path, Philox noise), MNIST softmax shape.  Usage: python tools/probe_batch.py [C ...] [f32]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
from dropout_hamiltonian_montecarlo_amd import _native as nat

dtype = torch.float32 if 'f32' in sys.argv else torch.float64
Cs = [int(a) for a in sys.argv[1:] if a.isdigit()] or [1, 16, 64, 256]
N, B, D, K = 60000, 500, 784, 10
dev = torch.device('cuda', 0)
X = torch.from_numpy(np.random.RandomState(0).rand(N, D)).to(dev, dtype)
Y = torch.from_numpy(np.eye(K)[np.random.RandomState(1).randint(0, K, N)]).to(dev, dtype)
ctx = nat.context(0)
ctx.set_sghmc_path(1)
eps, lam = 1e-3, 1e-2
for C in Cs:
    W = torch.zeros(D, C * K, dtype=dtype, device=dev)
    b = torch.zeros(C * K, dtype=dtype, device=dev)
    steps = 24
    rng = np.random.RandomState(5)
    L = np.ceil(2 * rng.rand(steps, C) * lam / eps)
    n_iter = np.maximum(0, np.ceil(L - 1)).astype(np.int32)
    u = rng.rand(steps, C)
    row0 = (np.arange(steps) % (N // B) * B).astype(np.int64)
    epsa = np.full(steps, eps)
    noff = np.zeros(steps * C, dtype=np.int64)
    out_A = torch.empty(steps * C, dtype=torch.float64, device=dev)
    out_acc = torch.empty(steps * C, dtype=torch.int32, device=dev)
    out_ll = torch.empty(steps * C, dtype=torch.float64, device=dev)
    a = nat.SamplerArgs()
    a.dtype = nat.dtype_code(dtype)
    a.B, a.D, a.K, a.C, a.n_steps = B, D, K, C, steps
    a.alpha, a.log_prior = 0.01, 0.0
    a.X, a.Y = nat.ptr(X), nat.ptr(Y)
    a.row0 = nat.addr(row0)
    a.eps = nat.addr(epsa)
    n_iter_f = np.ascontiguousarray(n_iter.reshape(-1))
    u_f = np.ascontiguousarray(u.reshape(-1))
    a.n_iter = nat.addr(n_iter_f)
    a.u_accept = nat.addr(u_f)
    a.noise_mode = nat.NOISE_PHILOX
    a.noise_off = nat.addr(noff)
    a.seed, a.chain0, a.step_base = 7, 0, 0
    a.W, a.b = nat.ptr(W), nat.ptr(b)
    a.out_A, a.out_accepted, a.out_ll = nat.ptr(out_A), nat.ptr(out_acc), nat.ptr(out_ll)
    ctx.check(ctx.lib.hmcx_sghmc_run(ctx.h, a), "warmup")
    torch.cuda.synchronize()
    ctx.set_timing(True)
    t0 = time.perf_counter()
    ctx.check(ctx.lib.hmcx_sghmc_run(ctx.h, a), "run")
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kms, kn = ctx.get_timing()
    ctx.set_timing(False)
    lf = float(n_iter.sum())
    maxit = float(n_iter.max(axis=1).sum())
    flop = 4.0 * B * D * K * C * maxit
    print("C=%4d %s steps %d lf %.0f (max-iter sum %.0f) wall %.4f s kern %.4f s  lf/s %.0f  lf/s*P %.3e  "
          "GEMM TFLOP/s %.2f  acc %.3f" % (C, 'f32' if dtype == torch.float32 else 'f64', steps, lf, maxit, dt,
                                           kms / 1e3, lf / dt, lf / dt * (D * K + K), flop / (kms / 1e3) / 1e12,
                                           out_acc.float().mean().item()), flush=True)
