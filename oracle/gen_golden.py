#!/usr/bin/env python3
"""ORACLE (test infrastructure only) — generate tests/golden/*.npz by running the
REFERENCE's own NumPy code (/root/reference, read-only) in a child process.

Run once in the build container:  ``python oracle/gen_golden.py`` (``--logistic``: only the
logistic-model / momentum-SGD fixtures of section 4; ``--notebook``: only the notebook-harness
fixture of section 5)
(the reference does not exist on the GPU box; the committed .npz files travel instead).

The reference needs a four-line import shim on Python 3.10 / NumPy 2:
``collections.Iterable`` (utils.py:2), ``h5py`` (imported but only used by HDF5
backends), ``np.int``/``np.float`` (utils.py:7).  SGHMC runs with the A1 completion
(SURVEY §8a): ``draw_momentum``/``accept``/``potential_energy`` taken from the
reference's own cpu/hmc.py, and ``sample`` fed the first two entries of step()'s
3-tuple.  Per-step integers are observed from the outside (grad-call counting and
array identity), without modifying the reference code path.
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, 'tests', 'golden')

CHILD = r'''
import sys, types, collections, collections.abc, io, contextlib, importlib.util, hashlib, json
sys.dont_write_bytecode = True
sys.path.insert(0, '/root/reference')
collections.Iterable = collections.abc.Iterable
sys.modules['h5py'] = types.ModuleType('h5py')
import numpy as np
np.int = int
np.float = float
spec = importlib.util.spec_from_file_location('golden_inputs', sys.argv[1])
gi = importlib.util.module_from_spec(spec); spec.loader.exec_module(gi)
OUT = sys.argv[2]

from hamiltonian.models.cpu.softmax import softmax as ref_softmax
from hamiltonian.models.cpu.mvn_gaussian import mvn_gaussian as ref_mvn
from hamiltonian.inference.cpu.sgld import sgld as ref_sgld
from hamiltonian.inference.cpu.sghmc import sghmc as ref_sghmc
from hamiltonian.inference.cpu import hmc as ref_hmc_mod
from hamiltonian.utils import one_hot as ref_one_hot

def sha(a):
    return hashlib.sha256(np.ascontiguousarray(np.asarray(a, dtype=np.float64)).tobytes()).hexdigest()

quiet = contextlib.redirect_stdout(io.StringIO())

# ---- (1) softmax grad / log_likelihood / nlp / log_prior --------------------------
out = {}
meta = {}
for i, (seed, B, ws) in enumerate(gi.GRAD_CASES):
    X, Y, W, b = gi.softmax_inputs(seed, B, wscale=ws)
    # cross-check the label encoding against the reference's utils.one_hot
    lab = Y.argmax(axis=1)
    assert np.array_equal(ref_one_hot(lab, 10), Y)
    m = ref_softmax({'alpha': 0.01})
    par = {'weights': W, 'bias': b}
    g = m.grad(par, X_train=X, y_train=Y)
    ll = m.log_likelihood(par, X_train=X, y_train=Y)
    nlp = m.negative_log_posterior(par, X_train=X, y_train=Y)
    lp = m.log_prior(par, X_train=X, y_train=Y)
    yhat = m.net(par, X)
    full = (seed, B, ws) in [(0, 32, 0.01), (0, 500, 0.01), (4, 64, 50.0), (5, 1, 0.01)]
    if full:
        out['c%d_gW' % i] = g['weights']
        out['c%d_yhat' % i] = yhat
    out['c%d_gW_slice' % i] = g['weights'][:8]
    out['c%d_gb' % i] = g['bias']
    out['c%d_scalars' % i] = np.array([ll, nlp, lp])
    meta['c%d' % i] = dict(seed=seed, B=B, wscale=ws, full=full,
                           gW_sha=sha(g['weights']), gb_sha=sha(g['bias']), yhat_sha=sha(yhat))
out['meta'] = np.array(json.dumps(meta))
np.savez_compressed(OUT + '/softmax_grad.npz', **out)

# ---- (2) SG-MCMC trajectories -----------------------------------------------------
class sghmc_completed(ref_sghmc):
    draw_momentum = ref_hmc_mod.hmc.draw_momentum
    accept = ref_hmc_mod.hmc.accept
    potential_energy = ref_hmc_mod.hmc.potential_energy
    def step(self, state, momentum, rng, **args):
        eps = self.step_size
        self._calls = 0
        q, p, A = ref_sghmc.step(self, state, momentum, rng, **args)
        n_iter = (self._calls - 1) // len(self.start)        # minus the dead grad at sghmc.py:26
        accepted = any(q[v] is not state[v] for v in state)
        self.rec.append((n_iter, float(A), int(accepted), eps))
        return q, p

class counting_model(ref_softmax):
    def __init__(self, hyper, owner):
        super().__init__(hyper); self.owner = owner
    def grad(self, par, **args):
        self.owner[0]._calls += 1
        return super().grad(par, **args)

class sgld_rec(ref_sgld):
    def step(self, state, momentum, rng, **args):
        self.rec.append((1, 1.0, 1, self.step_size))
        return ref_sgld.step(self, state, momentum, rng, **args)

for name, c in gi.TRAJ_CONFIGS.items():
    X, Y = gi.dataset(c['data_seed'], c['N'], c['D'], c['K'])
    owner = [None]
    model = counting_model({'alpha': c['alpha']}, owner)
    start = {'weights': np.zeros((c['D'], c['K'])), 'bias': np.zeros(c['K'])}
    cls = sghmc_completed if c['kind'] == 'sghmc' else sgld_rec
    s = cls(model, start, path_length=c['path_length'], step_size=c['step_size'], verbose=True)
    s.rec = []; s._calls = 0; owner[0] = s
    np.random.seed(c['np_seed'])
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf), contextlib.redirect_stderr(io.StringIO()):
        post, logp = s.sample(epochs=c['epochs'], burnin=c['burnin'], batch_size=c['B'],
                              rng=np.random.RandomState(c['rng_seed']), X_train=X, y_train=Y)
    rec = np.array(s.rec, dtype=np.float64)
    o = dict(logp=logp, trace=rec, log=np.array(buf.getvalue()))
    for v in post:
        o['post_' + v + '_sha'] = np.array(sha(post[v]))
        o['post_' + v + '_last'] = post[v][-1] if post[v][-1].size <= 1000 else post[v][-1][:16]
        if post[v].size <= 4000:
            o['post_' + v] = post[v]
        o['post_' + v + '_mean'] = post[v].reshape(post[v].shape[0], -1).mean(axis=1)
    np.savez_compressed(OUT + '/traj_%s.npz' % name, **o)

# ---- (3) full-batch HMC: MVN (config 1) and softmax -----------------------------------
c = gi.MVN_CONFIG
hyper = {'mu': np.array(c['mu']), 'cov': np.array(c['cov'])}
class hmc_rec(ref_hmc_mod.hmc):
    def step(self, state, momentum, rng, **args):
        eps = self.step_size
        self._calls = 0
        out = ref_hmc_mod.hmc.step(self, state, momentum, rng, **args)
        n_iter = (self._calls - 1) // len(self.start)
        accepted = any(out[0][v] is not state[v] for v in state)
        self.rec.append((n_iter, float(out[4]), int(accepted), eps))
        return out
class counting_mvn(ref_mvn):
    def grad(self, par, **args):
        self.owner._calls += 1
        return super().grad(par, **args)
m = counting_mvn(hyper)
h = hmc_rec(m, {'x': np.zeros(2)}, path_length=c['path_length'], step_size=c['step_size'], verbose=True)
m.owner = h; h.rec = []
np.random.seed(c['np_seed'])
with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
    post, loss, pos, mom = h.sample(c['niter'], c['burnin'], np.random.RandomState(c['rng_seed']))
np.savez_compressed(OUT + '/hmc_mvn.npz', post_x=post['x'], loss=loss,
                    trace=np.array(h.rec, dtype=np.float64),
                    pos0=np.array([p[0]['x'] for p in pos]), mom0=np.array([p[0]['x'] for p in mom]))

c = gi.HMC_SOFTMAX_CONFIG
X, Y = gi.dataset(c['data_seed'], c['N'], c['D'], c['K'])
class counting_softmax(ref_softmax):
    def grad(self, par, **args):
        self.owner._calls += 1
        return super().grad(par, **args)
m = counting_softmax({'alpha': c['alpha']})
h = hmc_rec(m, {'weights': np.zeros((c['D'], c['K'])), 'bias': np.zeros(c['K'])},
            path_length=c['path_length'], step_size=c['step_size'], verbose=True)
m.owner = h; h.rec = []
np.random.seed(c['np_seed'])
with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
    post, loss, pos, mom = h.sample(c['niter'], c['burnin'], np.random.RandomState(c['rng_seed']),
                                    X_train=X, y_train=Y)
np.savez_compressed(OUT + '/hmc_softmax.npz', post_weights=post['weights'], post_bias=post['bias'],
                    loss=loss, trace=np.array(h.rec, dtype=np.float64))
print('ok')
'''

# ---- (4) logistic model and momentum SGD: models/cpu/logistic.py,
# inference/cpu/sgd.py.  Separate child so the earlier fixtures are not rewritten.
CHILD_LOGISTIC = r'''
import sys, types, collections, collections.abc, io, contextlib, importlib.util, json
sys.dont_write_bytecode = True
sys.path.insert(0, '/root/reference')
collections.Iterable = collections.abc.Iterable
sys.modules['h5py'] = types.ModuleType('h5py')
import numpy as np
np.int = int
np.float = float
spec = importlib.util.spec_from_file_location('golden_inputs', sys.argv[1])
gi = importlib.util.module_from_spec(spec); spec.loader.exec_module(gi)
OUT = sys.argv[2]
from hamiltonian.models.cpu.logistic import logistic as ref_logistic
from hamiltonian.models.cpu.softmax import softmax as ref_softmax
from hamiltonian.inference.cpu.sgd import sgd as ref_sgd

out = {}
for i, (seed, B, D, ws) in enumerate(gi.LOGISTIC_CASES):
    X, y, W, b = gi.logistic_inputs(seed, B, D, wscale=ws)
    m = ref_logistic({'alpha': 0.25})
    par = {'weights': W, 'bias': b}
    g = m.grad(par, X_train=X, y_train=y)
    out['c%d_gW' % i] = g['weights']
    out['c%d_gb' % i] = g['bias']
    out['c%d_net' % i] = m.net(par, X_train=X)
    out['c%d_scalars' % i] = np.array([m.log_likelihood(par, X_train=X, y_train=y),
                                       m.negative_log_posterior(par, X_train=X, y_train=y),
                                       m.log_prior(par)])
    bs = max(1, B // 3)
    out['c%d_pred' % i] = m.predict(par, X, prob=False, batchsize=bs)
    out['c%d_predp' % i] = m.predict(par, X, prob=True, batchsize=bs)
np.savez_compressed(OUT + '/logistic.npz', **out)

for name, c in gi.SGD_CONFIGS.items():
    X, Y, start = gi.sgd_problem(c)
    model = ref_logistic({'alpha': c['alpha']}) if c['model'] == 'logistic' else ref_softmax({'alpha': c['alpha']})
    opt = ref_sgd(model, {k: v.copy() for k, v in start.items()}, step_size=c['step_size'])
    np.random.seed(c['np_seed'])
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        if c['dropout']:
            par, loss = opt.fit_dropout(epochs=c['epochs'], batch_size=c['B'], gamma=c['gamma'], p=c['p'],
                                        X_train=X, y_train=Y)
        else:
            par, loss = opt.fit(epochs=c['epochs'], batch_size=c['B'], gamma=c['gamma'], X_train=X, y_train=Y)
    np.savez_compressed(OUT + '/sgd_%s.npz' % name, weights=par['weights'], bias=par['bias'], loss=loss)
print('ok')
'''


# ---- (5) the notebook harness (benchmarks/1.-Simulated_data.ipynb cells 2, 6, 10) through the
# reference's own import paths hamiltonian.models.cpu.logistic / inference.cpu.sgd / inference.cpu.hmc.
CHILD_NOTEBOOK = r'''
import sys, types, collections, collections.abc, io, contextlib, importlib.util
sys.dont_write_bytecode = True
sys.path.insert(0, '/root/reference')
collections.Iterable = collections.abc.Iterable
sys.modules['h5py'] = types.ModuleType('h5py')
import numpy as np
np.int = int
np.float = float
spec = importlib.util.spec_from_file_location('golden_inputs', sys.argv[1])
gi = importlib.util.module_from_spec(spec); spec.loader.exec_module(gi)
OUT = sys.argv[2]
import hamiltonian.models.cpu.logistic as base_model_cpu
import hamiltonian.inference.cpu.sgd as inference_cpu
import hamiltonian.inference.cpu.hmc as sampler_cpu

X_train, X_test, y_train, y_test = gi.notebook_data()
c = gi.NOTEBOOK['sgd']
D = X_train.shape[1]
np.random.seed(c['start_seed'])
start_p = {'weights': 2 * np.random.random((D, 1)), 'bias': 2 * np.random.random(1)}
hyper_p = {'alpha': c['alpha']}
model_cpu = base_model_cpu.logistic(hyper_p)
optim_cpu = inference_cpu.sgd(model_cpu, {k: v.copy() for k, v in start_p.items()}, step_size=c['eta'])
with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
    par_cpu, loss = optim_cpu.fit(epochs=c['epochs'], batch_size=c['batch_size'], gamma=c['gamma'],
                                  X_train=X_train, y_train=y_train, verbose=True)
y_pred = model_cpu.predict(par_cpu, X_test, batchsize=c['batch_size'])

h = gi.NOTEBOOK['hmc']
class rec(sampler_cpu.hmc):
    def step(self, state, momentum, rng, **args):
        self._calls = 0
        out = sampler_cpu.hmc.step(self, state, momentum, rng, **args)
        n_iter = (self._calls - 1) // len(self.start)
        accepted = any(out[0][v] is not state[v] for v in state)
        self.rec.append((n_iter, float(out[4]), int(accepted)))
        return out
class counting(base_model_cpu.logistic):
    def grad(self, par, **args):
        self.owner._calls += 1
        return super().grad(par, **args)
m = counting(hyper_p)
s = rec(m, start_p, path_length=h['path_length'], step_size=h['step_size'])
m.owner = s; s.rec = []
np.random.seed(h['np_seed'])
with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
    samples, hloss, positions, momentums = s.sample(h['niter'], h['burnin'], np.random.RandomState(h['rng_seed']),
                                                    X_train=X_train, y_train=y_train)
par_mean = {var: np.mean(samples[var], axis=0).reshape(start_p[var].shape) for var in samples.keys()}
np.savez_compressed(OUT + '/notebook_simulated.npz', X_train=X_train, y_train=y_train, X_test=X_test, y_test=y_test,
                    start_weights=start_p['weights'], start_bias=start_p['bias'],
                    sgd_weights=par_cpu['weights'], sgd_bias=par_cpu['bias'], sgd_loss=loss, sgd_pred=y_pred,
                    hmc_weights=samples['weights'], hmc_bias=samples['bias'], hmc_loss=hloss,
                    hmc_trace=np.array(s.rec, dtype=np.float64),
                    hmc_mom0=np.array([np.concatenate([p[0]['weights'].ravel(), p[0]['bias'].ravel()]) for p in momentums]),
                    hmc_pred=model_cpu.predict(par_mean, X_test, batchsize=c['batch_size']))
print('ok')
'''


def _run_child(code, env):
    r = subprocess.run([sys.executable, '-c', code, os.path.join(REPO, 'oracle', 'inputs.py'), OUT],
                       env=env, capture_output=True, text=True)
    sys.stdout.write(r.stdout[-2000:])
    sys.stderr.write(r.stderr[-4000:])
    if r.returncode != 0:
        raise SystemExit(r.returncode)


def main():
    os.makedirs(OUT, exist_ok=True)
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE='1', OPENBLAS_NUM_THREADS='1')
    if '--logistic' in sys.argv:            # only the logistic / sgd fixtures (4)
        _run_child(CHILD_LOGISTIC, env)
        return
    if '--notebook' in sys.argv:            # only the notebook-harness fixture (5)
        _run_child(CHILD_NOTEBOOK, env)
        return
    r = subprocess.run([sys.executable, '-c', CHILD, os.path.join(REPO, 'oracle', 'inputs.py'), OUT],
                       env=env, capture_output=True, text=True)
    sys.stdout.write(r.stdout[-2000:])
    sys.stderr.write(r.stderr[-4000:])
    if r.returncode != 0:
        raise SystemExit(r.returncode)
    info = {'generator': 'oracle/gen_golden.py', 'reference': '/root/reference (read-only)',
            'numpy': __import__('numpy').__version__, 'OPENBLAS_NUM_THREADS': 1}
    with open(os.path.join(OUT, 'PROVENANCE.json'), 'w') as f:
        json.dump(info, f, indent=1)


if __name__ == '__main__':
    main()
