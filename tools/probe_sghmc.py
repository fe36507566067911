"""Quick timing probe: SGHMC softmax (B=500, D=784, K=10) in philox mode on cuda:0."""
import io
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.softmax import softmax
from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.sghmc import sghmc

dtype = torch.float32 if (len(sys.argv) > 1 and sys.argv[1] == 'f32') else torch.float64
graph = len(sys.argv) > 2 and sys.argv[2] == 'graph'
N = 12000
X = np.random.RandomState(0).rand(N, 784)
Y = np.eye(10)[np.random.RandomState(1).randint(0, 10, N)]
m = softmax({'alpha': 0.01}, dtype=dtype)
if graph:
    m.ctx.set_graph_mode(True)
s = sghmc(m, {'weights': np.zeros((784, 10)), 'bias': np.zeros(10)}, path_length=1e-2, step_size=1e-3,
          noise='philox', seed=1)
s.out = io.StringIO()
s.trace = []
s.sample(epochs=1, burnin=0, batch_size=500, X_train=X, y_train=Y)   # warm-up
torch.cuda.synchronize()
s.trace = []
t0 = time.perf_counter()
s.sample(epochs=2, burnin=0, batch_size=500, X_train=X, y_train=Y)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
lf = sum(max(0, t['L'] - 1) for t in s.trace)
print('dtype', dtype, 'graph', graph, 'steps', len(s.trace), 'leapfrogs', lf, 'time %.4f s' % dt,
      'lf/s %.1f' % (lf / dt), 'us/lf %.2f' % (dt / lf * 1e6), 'acc', np.mean([t['accepted'] for t in s.trace]))
