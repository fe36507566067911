"""Micro-timings of the host operations on the sampler's call path (µs per op, median of 2000)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
from dropout_hamiltonian_montecarlo_amd import _native as nat

dev = torch.device("cuda:0")
ctx = nat.context(dev)
d = torch.empty(1 << 16, dtype=torch.uint8, device=dev)
h = torch.empty(1 << 16, dtype=torch.uint8, pin_memory=True)
ev = torch.cuda.Event()
eps = [1e-3] * 20
rows = list(range(0, 10000, 500))


def t(name, fn, n=2000):
    for _ in range(50):
        fn()
    v = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        v.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    print("%-40s %7.2f us" % (name, np.median(v) * 1e6))


t("nat.context(dev)", lambda: nat.context(dev))
t("torch.cuda.current_stream()", lambda: torch.cuda.current_stream())
t("ev.record()", lambda: ev.record())
t("ev.synchronize() (done)", lambda: ev.synchronize())
t("h[:724].copy_(d[:724], non_blocking)", lambda: h[:724].copy_(d[:724], non_blocking=True))
t("philox_schedule(20)", lambda: nat.philox_schedule(1, 0, 1, 0, 1e-2, eps))
t("SamplerArgs() + 30 fields", lambda: [setattr(nat.SamplerArgs(), "B", 1) for _ in range(30)])
t("np.asarray(rows, int64)", lambda: np.asarray(rows, dtype=np.int64))
t("ptr(d)", lambda: nat.ptr(d))
t("h[:724].numpy().copy()", lambda: h[:724].numpy().copy())
t("torch.cuda.synchronize()", lambda: torch.cuda.synchronize())
t("torch.cuda.is_available()", lambda: torch.cuda.is_available(), n=200)
