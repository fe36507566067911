"""Host path of one driver-shape call (bench.py --steps 20): enqueue (Python + C call), kernel
(context HIP events), and the end of the timed region two ways — torch.cuda.synchronize() straight
away, or first spinning on the verdict word the kernel writes into the pinned host block.
    python tools/probe_hostpath.py [steps=20] [reps=40]"""
import io
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.softmax import softmax
from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu import sghmc as sgmod

kw = dict(a.split('=') for a in sys.argv[1:] if '=' in a)
n_steps, reps = int(kw.get('steps', 20)), int(kw.get('reps', 40))
N, B = 60000, 500
X = np.random.RandomState(0).rand(N, 784)
Y = np.eye(10)[np.random.RandomState(1).randint(0, 10, N)]
m = softmax({'alpha': 0.01}, dtype=torch.float64)
s = sgmod.sghmc(m, {'weights': np.zeros((784, 10)), 'bias': np.zeros(10)}, path_length=1e-2, step_size=1e-3,
                noise='philox', seed=1)
s.out = io.StringIO()
data = s._upload_data(X, Y)
state = s._init_state()
lib = m.ctx.lib
crun_t = []
orig = lib.hmcx_sghmc_run


def crun(h, a):
    t = time.perf_counter(); r = orig(h, a); crun_t.append(time.perf_counter() - t); return r


lib.hmcx_sghmc_run = crun
nb = N // B
res = {k: [] for k in ('enqueue', 'ccall', 'kernel', 'wall_sync', 'wall_spin', 'spin_seen', 'sync_after_spin')}
step = 0
for i in range(2 * reps + 4):
    spin = i % 2 == 1
    rows = [((step + j) % nb) * B for j in range(n_steps)]
    step += n_steps
    s.trace = None
    m.ctx.set_timing(True)
    torch.cuda.synchronize()
    ring = s.__dict__.get('_io_ring')
    if ring is not None:
        slot = ring[s._io_next % s._IO_SLOTS]
        slot['hnp'][36 * n_steps:36 * n_steps + 4].view(np.int32)[0] = -7
    t0 = time.perf_counter()
    h = s._enqueue(state, data, rows, [1e-3] * n_steps, None, B)
    t1 = time.perf_counter()
    if spin:
        w = h['hnp'][36 * n_steps:36 * n_steps + 4].view(np.int32)
        while w[0] == -7:
            pass
        t2 = time.perf_counter()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    s._collect(h)
    kms, _ = m.ctx.get_timing()
    m.ctx.set_timing(False)
    if i < 4:
        continue
    res['enqueue'].append(t1 - t0)
    res['ccall'].append(crun_t[-1])
    res['kernel'].append(kms * 1e-3)
    if spin:
        res['wall_spin'].append(t3 - t0)
        res['spin_seen'].append(t2 - t0)
        res['sync_after_spin'].append(t3 - t2)
    else:
        res['wall_sync'].append(t3 - t0)
for k, v in res.items():
    v = np.array(v) * 1e6
    print('%-16s median %8.1f us  min %8.1f  max %8.1f' % (k, np.median(v), v.min(), v.max()))
k = np.median(res['kernel']) * 1e6
print('overhead (wall - kernel): sync %.1f us, spin %.1f us' % (np.median(res['wall_sync']) * 1e6 - k,
                                                                 np.median(res['wall_spin']) * 1e6 - k))
