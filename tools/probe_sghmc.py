"""Quick timing probe: SGHMC softmax (B=500, D=784, K=10) in philox mode on cuda:0."""
import ctypes
import io
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
from dropout_hamiltonian_montecarlo_amd import _native as nat
from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.softmax import softmax
from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.sghmc import sghmc

dtype = torch.float32 if 'f32' in sys.argv else torch.float64
graph = 'graph' in sys.argv
N = 60000
X = np.random.RandomState(0).rand(N, 784)
Y = np.eye(10)[np.random.RandomState(1).randint(0, 10, N)]
m = softmax({'alpha': 0.01}, dtype=dtype)
m.ctx.set_graph_mode(graph)
m.ctx.set_sghmc_path(1 if 'kern' in sys.argv else 0)
s = sghmc(m, {'weights': np.zeros((784, 10)), 'bias': np.zeros(10)}, path_length=1e-2, step_size=1e-3,
          noise='philox', seed=1)
s.out = io.StringIO()
s.trace = []
s.sample(epochs=1, burnin=0, batch_size=500, X_train=X, y_train=Y)   # warm-up
torch.cuda.synchronize()
# time the raw C-ABI call for one epoch (schedule prepared outside the timed region)
data = s._upload_data(X, Y)
state = s._init_state()
rows = list(range(0, N - 500 + 1, 500))
eps = [1e-3] * len(rows)
orig = nat.context
t_host = []
_lib_run = m.ctx.lib.hmcx_sghmc_run
def timed_run(h, a):
    t0 = time.perf_counter(); rc = _lib_run(h, a); t_host.append(time.perf_counter() - t0); return rc
class L: pass
reps = int([a for a in sys.argv if a.startswith('reps=')][0][5:]) if any(a.startswith('reps=') for a in sys.argv) else 5
m.ctx.lib.hmcx_sghmc_run = timed_run
dts, lfs = [], []
try:
    for _ in range(reps):
        s.trace = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = s._run(state, data, rows, eps, None, 500)
        torch.cuda.synchronize()
        dts.append(time.perf_counter() - t0)
        lfs.append(sum(max(0, t['L'] - 1) for t in s.trace))
finally:
    m.ctx.lib.hmcx_sghmc_run = _lib_run
us = sorted(d / l * 1e6 for d, l in zip(dts, lfs))
dt, lf = dts[-1], lfs[-1]
print('dtype', dtype, 'graph', graph, 'kern' in sys.argv, 'steps', len(s.trace), 'leapfrogs', lf, 'wall %.4f s' % dt,
      'enqueue %.4f s' % t_host[0], 'lf/s %.1f' % (lf / dt), 'us/lf %.2f' % us[len(us) // 2],
      'min %.2f max %.2f' % (us[0], us[-1]), 'acc %.3f' % np.mean(res.accepted), flush=True)
