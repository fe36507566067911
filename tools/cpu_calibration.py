#!/usr/bin/env python3
"""CPU-port calibration (BASELINE.md:45): how fast the oracle's restatement of the
reference SGHMC (oracle/samplers.py, what bench.py's `cpu_baseline` legs time on the GPU box) runs
against the reference's own NumPy code (/root/reference, read-only, with the import shim of
oracle/gen_golden.py) on the same loop, same minibatches, same seeds.

Run in the build container (the reference does not exist on the GPU box):

    python tools/cpu_calibration.py [--seconds 10]

For each BLAS thread count (1, and every CPU of this container) one child process times both
implementations in alternating rounds (≥ `--seconds` each): `sample(epochs=1, burnin=0,
batch_size=500)` over 10 minibatches of the bench's synthetic MNIST-shaped data (D=784, K=10,
α=0.01, ε=1e-3, λ=1e-2), leapfrogs counted as bench.py counts them (L−1 per step; the reference's
dead gradient at sghmc.py:26 is part of its time, not of its leapfrog count).  Writes
profiles/cpu_calibration.json; bench.py copies `ratio_port_over_reference` of the matching thread
count into each cpu_baseline line as `calibration_ratio`.
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "profiles", "cpu_calibration.json")

CHILD = r'''
import sys, types, collections, collections.abc, io, contextlib, time, json
sys.dont_write_bytecode = True
REPO, SECONDS = sys.argv[1], float(sys.argv[2])
sys.path.insert(0, '/root/reference')
collections.Iterable = collections.abc.Iterable
sys.modules['h5py'] = types.ModuleType('h5py')
import numpy as np
np.int = int
np.float = float
from hamiltonian.models.cpu.softmax import softmax as ref_softmax
from hamiltonian.inference.cpu.sghmc import sghmc as ref_sghmc
from hamiltonian.inference.cpu import hmc as ref_hmc_mod
sys.path.insert(0, REPO)
from oracle import models as om, samplers as osm

D, K, B, NB = 784, 10, 500, 10
ALPHA, EPS, LAMBDA = 0.01, 1e-3, 1e-2
X = np.random.RandomState(0).rand(NB * B, D)
lab = np.random.RandomState(1).randint(0, K, NB * B)
Y = np.zeros((NB * B, K)); Y[np.arange(NB * B), lab] = 1.0

class ref_completed(ref_sghmc):
    # A1 completion (SURVEY §8a), exactly as oracle/gen_golden.py runs the reference
    draw_momentum = ref_hmc_mod.hmc.draw_momentum
    accept = ref_hmc_mod.hmc.accept
    potential_energy = ref_hmc_mod.hmc.potential_energy
    def step(self, state, momentum, rng, **args):
        q, p, A = ref_sghmc.step(self, state, momentum, rng, **args)
        return q, p

def run_ref(rep):
    s = ref_completed(ref_softmax({'alpha': ALPHA}), {'weights': np.zeros((D, K)), 'bias': np.zeros(K)},
                      path_length=LAMBDA, step_size=EPS, verbose=False)
    np.random.seed(rep)
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        s.sample(epochs=1, burnin=0, batch_size=B, rng=np.random.RandomState(rep), X_train=X, y_train=Y)
    return time.perf_counter() - t0

def run_port(rep):
    s = osm.sghmc(om.softmax({'alpha': ALPHA}), {'weights': np.zeros((D, K)), 'bias': np.zeros(K)},
                  path_length=LAMBDA, step_size=EPS, verbose=False)
    s.out = io.StringIO(); s.trace = []
    np.random.seed(rep)
    t0 = time.perf_counter()
    post, _ = s.sample(epochs=1, burnin=0, batch_size=B, rng=np.random.RandomState(rep), X_train=X, y_train=Y)
    dt = time.perf_counter() - t0
    return dt, sum(max(0.0, t['L'] - 1) for t in s.trace), post

tot = {'reference': [0.0, 0.0, 0], 'port': [0.0, 0.0, 0]}
rep = 0
same = True
while min(tot['reference'][0], tot['port'][0]) < SECONDS:
    dt_p, lf, post = run_port(rep)
    dt_r = run_ref(rep)
    tot['port'][0] += dt_p; tot['port'][1] += lf; tot['port'][2] += 1
    # the reference consumes the same global/sampler streams in the same order (bit-exact parity,
    # tests/test_oracle_golden.py), so its leapfrog count per call equals the port's
    tot['reference'][0] += dt_r; tot['reference'][1] += lf; tot['reference'][2] += 1
    rep += 1
import threadpoolctl
thr = max((i.get('num_threads', 1) for i in threadpoolctl.threadpool_info() if i.get('user_api') == 'blas'), default=1)
print(json.dumps({'blas_threads': int(thr), 'calls': rep,
                  'reference': {'seconds': tot['reference'][0], 'leapfrogs': tot['reference'][1],
                                'lf_per_s': tot['reference'][1] / tot['reference'][0]},
                  'port': {'seconds': tot['port'][0], 'leapfrogs': tot['port'][1],
                           'lf_per_s': tot['port'][1] / tot['port'][0]}}))
'''


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    args = ap.parse_args()
    if not os.path.isdir("/root/reference"):
        sys.exit("cpu_calibration: /root/reference is absent (run this in the build container)")
    ncpu = len(os.sched_getaffinity(0))
    res = {}
    for thr in sorted({1, ncpu}):
        env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", OPENBLAS_NUM_THREADS=str(thr),
                   OMP_NUM_THREADS=str(thr))
        r = subprocess.run([sys.executable, "-c", CHILD, REPO, str(args.seconds)], env=env,
                           capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stderr[-4000:])
            sys.exit(r.returncode)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        d["ratio_port_over_reference"] = d["port"]["lf_per_s"] / d["reference"]["lf_per_s"]
        res[str(d["blas_threads"])] = d
        print("threads %d: reference %.1f lf/s, port %.1f lf/s, ratio %.3f" % (
            d["blas_threads"], d["reference"]["lf_per_s"], d["port"]["lf_per_s"], d["ratio_port_over_reference"]))
    out = {"generator": "tools/cpu_calibration.py",
           "what": "oracle/samplers.py SGHMC (the bench's cpu_baseline 'port') vs the reference's own "
                   "hamiltonian/inference/cpu/sghmc.py + models/cpu/softmax.py (A1 completion, import shim of "
                   "oracle/gen_golden.py), same loop: sample(epochs=1, burnin=0, batch_size=500) over 10 "
                   "minibatches, D=784, K=10, alternating calls, leapfrogs = sum(L-1)",
           "host": cpu_model(), "cpus_in_mask": ncpu, "date": time.strftime("%Y-%m-%d"),
           "by_threads": res}
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", os.path.relpath(OUT, REPO))


if __name__ == "__main__":
    main()
