"""Fixed cost of one persistent SGHMC launch: kernel time (context HIP events) of one call of n steps
for n in 1 … 120, regressed on the call's leapfrog count and step count — the intercept is what a
launch costs beyond its steps.  Also the host enqueue time of each call.
    python tools/probe_launch_fixed.py [reps=6]"""
import io
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.softmax import softmax
from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu import sghmc as sgmod

kw = dict(a.split('=') for a in sys.argv[1:] if '=' in a)
reps = int(kw.get('reps', 6))
N, B = 60000, 500
X = np.random.RandomState(0).rand(N, 784)
Y = np.eye(10)[np.random.RandomState(1).randint(0, 10, N)]
m = softmax({'alpha': 0.01}, dtype=torch.float64)
s = sgmod.sghmc(m, {'weights': np.zeros((784, 10)), 'bias': np.zeros(10)}, path_length=1e-2, step_size=1e-3,
                noise='philox', seed=1)
s.out = io.StringIO()
data = s._upload_data(X, Y)
state = s._init_state()
nb = N // B
step = 0
rowsum = []
for n_steps in [5, 1, 2, 5, 10, 20, 40, 120] * reps:
    rows = [((step + i) % nb) * B for i in range(n_steps)]
    step += n_steps
    s.trace = None
    m.ctx.set_timing(True)
    torch.cuda.synchronize()
    time.sleep(0.002)
    t0 = time.perf_counter()
    h = s._enqueue(state, data, rows, [1e-3] * n_steps, None, B)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    res = s._collect(h)
    kms, _ = m.ctx.get_timing()
    m.ctx.set_timing(False)
    lf = float(np.maximum(0, np.asarray(res.L) - 1).sum())
    rowsum.append((n_steps, lf, kms * 1e3, (t1 - t0) * 1e6, (t2 - t0) * 1e6))
rs = np.array(rowsum[1:])
for n in sorted(set(rs[:, 0])):
    r = rs[rs[:, 0] == n]
    print('steps %4d  lf %7.1f  kernel %8.1f us  (%.3f us/lf)  enqueue %5.1f us  wall %8.1f us' % (
        n, r[:, 1].mean(), r[:, 2].mean(), r[:, 2].sum() / r[:, 1].sum(), np.median(r[:, 3]), r[:, 4].mean()))
A = np.c_[np.ones(len(rs)), rs[:, 0], rs[:, 1]]
coef, *_ = np.linalg.lstsq(A, rs[:, 2], rcond=None)
print('kernel us = %.1f + %.2f * steps + %.3f * leapfrogs' % tuple(coef))
A = np.c_[np.ones(len(rs)), rs[:, 1]]
coef, *_ = np.linalg.lstsq(A, rs[:, 2], rcond=None)
print('kernel us = %.1f + %.3f * leapfrogs' % tuple(coef))
