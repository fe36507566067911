"""Per-call host overhead of the headline sampler call (bench.py's timed region at --steps 20):
splits one enqueue/collect pair into its host phases and compares the wall time with the kernel
time the context's HIP events report.  python tools/probe_overhead.py [steps=20] [reps=50]"""
import io
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
from dropout_hamiltonian_montecarlo_amd import _native as nat
from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.softmax import softmax
from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu import sghmc as sgmod

kw = dict(a.split('=') for a in sys.argv[1:] if '=' in a)
n_steps, reps = int(kw.get('steps', 20)), int(kw.get('reps', 50))
N, B = 60000, 500
X = np.random.RandomState(0).rand(N, 784)
Y = np.eye(10)[np.random.RandomState(1).randint(0, 10, N)]
m = softmax({'alpha': 0.01}, dtype=torch.float64)
s = sgmod.sghmc(m, {'weights': np.zeros((784, 10)), 'bias': np.zeros(10)}, path_length=1e-2, step_size=1e-3,
                noise='philox', seed=1)
s.out = io.StringIO()
data = s._upload_data(X, Y)
state = s._init_state()
rows = [i * B for i in range(n_steps)]
eps = [1e-3] * n_steps
tm = {k: [] for k in ('sched', 'ccall', 'enqueue', 'collect', 'wall', 'kernel')}
orig_sched, lib_run = s._schedule, m.ctx.lib.hmcx_sghmc_run


def sched(*a):
    t = time.perf_counter(); r = orig_sched(*a); tm['sched'].append(time.perf_counter() - t); return r


def crun(h, a):
    t = time.perf_counter(); r = lib_run(h, a); tm['ccall'].append(time.perf_counter() - t); return r


s._schedule = sched
m.ctx.lib.hmcx_sghmc_run = crun
for i in range(reps + 5):
    s.trace = []
    m.ctx.set_timing(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    h = s._enqueue(state, data, rows, eps, None, B)
    t1 = time.perf_counter()
    s._collect(h)
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    kms, _ = m.ctx.get_timing()
    m.ctx.set_timing(False)
    if i >= 5:
        tm['enqueue'].append(t1 - t0); tm['collect'].append(t2 - t1); tm['wall'].append(t3 - t0)
        tm['kernel'].append(kms * 1e-3)
for k in tm:
    v = np.array(tm[k][-reps:]) * 1e6
    print('%-8s median %8.1f us  min %8.1f' % (k, np.median(v), v.min()))
print('overhead (wall - kernel) median %.1f us' % (np.median(np.array(tm['wall'][-reps:]) - np.array(tm['kernel'][-reps:])) * 1e6))
