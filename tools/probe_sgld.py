"""Timing probe: SGLD (config 5 shape: PlantVillage-like features D=2048, K=38, batch 500, one chain)
through hmcx_sgld_run with Philox noise.  Usage: python tools/probe_sgld.py [f32] [steps] [C]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
from dropout_hamiltonian_montecarlo_amd import _native as nat  # noqa: E402

dtype = torch.float32 if 'f32' in sys.argv else torch.float64
nums = [int(a) for a in sys.argv[1:] if a.isdigit()]
steps = nums[0] if nums else 200
C = nums[1] if len(nums) > 1 else 1
N, B, D, K = (60000, 500, 784, 10) if 'mnist' in sys.argv else (20000, 500, 2048, 38)
dev = torch.device('cuda', 0)
X = torch.from_numpy(np.random.RandomState(0).rand(N, D)).to(dev, dtype)
Y = torch.from_numpy(np.eye(K)[np.random.RandomState(1).randint(0, K, N)]).to(dev, dtype)
ctx = nat.context(0)
if 'graph' in sys.argv:
    ctx.set_graph_mode(True)
W = torch.zeros(D, C * K, dtype=dtype, device=dev)
b = torch.zeros(C * K, dtype=dtype, device=dev)
row0 = (np.arange(steps) % (N // B) * B).astype(np.int64)
epsa = np.full(steps, 1e-4)
want = np.zeros(steps, dtype=np.uint8)
want[::10] = 1
noff = np.zeros(steps * C, dtype=np.int64)
out_ll = torch.zeros(steps * C, dtype=torch.float64, device=dev)
a = nat.SamplerArgs()
a.dtype = nat.dtype_code(dtype)
a.B, a.D, a.K, a.C, a.n_steps = B, D, K, C, steps
a.alpha, a.log_prior = 0.01, 0.0
a.X, a.Y = nat.ptr(X), nat.ptr(Y)
a.row0 = nat.addr(row0)
a.eps = nat.addr(epsa)
a.want_ll = nat.addr(want)
a.noise_mode = nat.NOISE_PHILOX
a.noise_off = nat.addr(noff)
a.seed, a.chain0, a.step_base = 3, 0, 0
a.W, a.b = nat.ptr(W), nat.ptr(b)
a.out_ll = nat.ptr(out_ll)
ctx.check(ctx.lib.hmcx_sgld_run(ctx.h, a), "warmup")
torch.cuda.synchronize()
ctx.set_timing(True)
t0 = time.perf_counter()
ctx.check(ctx.lib.hmcx_sgld_run(ctx.h, a), "run")
torch.cuda.synchronize()
dt = time.perf_counter() - t0
kms, _ = ctx.get_timing()
ctx.set_timing(False)
P = D * K + K
flop = 4.0 * B * D * K * C * steps
print("SGLD %s C=%d steps %d wall %.4f s kern %.4f s  us/step %.2f  lf/s %.0f  lf/s*P %.3e  TFLOP/s %.2f  "
      "X GB/s %.0f  ll %.4f" % ('f64' if dtype == torch.float64 else 'f32', C, steps, dt, kms / 1e3, kms * 1e3 / steps,
                                steps * C / (kms / 1e3), steps * C / (kms / 1e3) * P, flop / (kms / 1e3) / 1e12,
                                B * D * X.element_size() * steps / (kms / 1e3) / 1e9, out_ll[-10].item()), flush=True)
