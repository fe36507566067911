"""Timing probe: config 3 (MNIST MLP 784-256-256-10, B = 500) SGHMC through hmcx_mlp_sghmc_run,
Philox noise and masks.  Usage: python tools/probe_mlp.py [f64] [steps] [lam=<path length>] [reps=<n>]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
from dropout_hamiltonian_montecarlo_amd import _native as nat  # noqa: E402

dtype = torch.float64 if 'f64' in sys.argv else torch.float32
steps = next((int(a) for a in sys.argv[1:] if a.isdigit()), 20)
N, B, n_in, n_mid, n_out = 60000, 500, 784, 256, 10
dev = torch.device('cuda', 0)
X = torch.from_numpy(np.random.RandomState(0).rand(N, n_in)).to(dev, dtype)
y = torch.from_numpy(np.random.RandomState(1).randint(0, n_out, N)).to(dev, torch.int32)
rs = np.random.RandomState(2)
shapes = [(n_mid, n_in), (n_mid,), (n_mid, n_mid), (n_mid,), (n_out, n_mid), (n_out,)]
par = [torch.from_numpy(rs.normal(0, 0.05, s)).to(dev, dtype).contiguous() for s in shapes]
P = sum(int(np.prod(s)) for s in shapes)
ctx = nat.context(0)
if 'graph' in sys.argv:
    ctx.set_graph_mode(True)
eps = 1e-3
lam = next((float(a[4:]) for a in sys.argv[1:] if a.startswith('lam=')), 5e-3)
reps = next((int(a[5:]) for a in sys.argv[1:] if a.startswith('reps=')), 1)
L = np.ceil(2 * rs.rand(steps) * lam / eps)
n_iter = np.maximum(0, np.ceil(L - 1)).astype(np.int32)
u = rs.rand(steps)
row0 = (np.arange(steps) % (N // B) * B).astype(np.int64)
epsa = np.full(steps, eps)
zoff = np.zeros(steps, dtype=np.int64)
out = [torch.empty(steps * w, dtype=torch.float64, device=dev) for w in (1, 1, 1, 2)]
out_acc = torch.empty(steps, dtype=torch.int32, device=dev)
a = nat.MlpSghmcArgs()
a.dtype = nat.dtype_code(dtype)
a.B, a.n_in, a.n_mid, a.n_out, a.n_steps = B, n_in, n_mid, n_out, steps
for i in range(6):
    a.order[i] = i
a.alpha = 0.01
a.X, a.y = nat.ptr(X), nat.ptr(y)
a.row0 = row0.ctypes.data_as(nat.c_i64p)
a.eps = epsa.ctypes.data_as(nat.c_dblp)
a.n_iter = n_iter.ctypes.data_as(nat.c_i32p)
a.u_accept = u.ctypes.data_as(nat.c_dblp)
a.noise_mode = a.mask_mode = nat.NOISE_PHILOX
a.noise_off = a.mask_off = zoff.ctypes.data_as(nat.c_i64p)
a.seed, a.chain, a.step_base = 5, 0, 0
for i in range(6):
    a.par.p[i] = par[i].data_ptr()
a.out_A, a.out_accepted = nat.ptr(out[0]), nat.ptr(out_acc)
a.out_loss, a.out_nlp, a.out_E = nat.ptr(out[1]), nat.ptr(out[2]), nat.ptr(out[3])
ctx.check(ctx.lib.hmcx_mlp_sghmc_run(ctx.h, a), "warmup")
torch.cuda.synchronize()
ctx.set_timing(True)
t0 = time.perf_counter()
for _ in range(reps):
    ctx.check(ctx.lib.hmcx_mlp_sghmc_run(ctx.h, a), "run")
torch.cuda.synchronize()
dt = time.perf_counter() - t0
kms, _ = ctx.get_timing()
ctx.set_timing(False)
lf = float(n_iter.sum()) * reps
# FLOP per leapfrog iteration (6 sub-steps, minimal recompute): forwards + backward parts
f_l1 = 2.0 * B * n_in * n_mid
f_l2 = 2.0 * B * n_mid * n_mid
f_l3 = 2.0 * B * n_mid * n_out
fwd_full = f_l1 + f_l2 + f_l3
per_iter = (2 * fwd_full + 4 * (f_l2 + f_l3)            # sub-steps W1, b1: full forward
            + (f_l3 + f_l2 + f_l2 + f_l2)               # W2: fwd (l2, l3) + ga2 + gW2  (approx.)
            + (f_l3 + f_l2 + f_l2)                      # b2
            + 2 * (f_l2 + f_l3 + f_l3)                  # W3, b3
            + 2 * (f_l2 + f_l1))                        # W1/b1 backward: ga1 + gW1
print("lam %g E[L-1] %.1f " % (lam, lf / steps / reps), end="")
print("MLP %s%s steps %d lf %.0f wall %.4f s kern %.4f s  lf/s %.1f  lf/s*P %.3e  ~GFLOP/s %.1f  acc %.3f  loss %.4f"
      % ('f64' if dtype == torch.float64 else 'f32', ' graph' if 'graph' in sys.argv else '', steps, lf, dt, kms / 1e3, lf / (kms / 1e3),
         lf / (kms / 1e3) * P, per_iter * lf / (kms / 1e3) / 1e9, out_acc.float().mean().item(),
         out[1][-1].item()), flush=True)
