"""MNIST HDF5 loader — the data step before the sampler in the reference's MNIST benchmark.

Reference: /root/reference/benchmarks/2.-MNIST.ipynb cell 2: ``mnist_train.h5`` holds
``X_train`` [N, 28, 28] and ``y_train`` [N] (``mnist_test.h5``: ``X_test``, ``y_test``);
X is flattened to [N, 784] and divided by 255., K = len(np.unique(y_train)), and labels become
one_hot(y, K) (utils.py:4-8).  Read through the HDF5 C library (h5trace; h5py is not in this
image).  ``device=`` additionally returns the arrays resident on the GPU as torch tensors of
``dtype`` (the samplers upload once per ``sample`` call anyway; this keeps one copy in HBM for
repeated calls).
"""
import os

import numpy as np

from dropout_hamiltonian_montecarlo_amd import h5trace

from .utils import one_hot


def load_mnist(data_path, device=None, dtype=None):
    """Returns X_train, y_train, X_test, y_test exactly as the notebook builds them (float64,
    one-hot labels); with ``device`` the four are torch tensors on that device."""
    def read(fname, xname, yname):
        path = os.path.join(data_path, fname)
        X = h5trace.read_dataset(path, xname, dtype=np.float64)        # uint8 → float64 is exact
        X = X.reshape((-1, 28 * 28))
        X = X / 255.
        y = h5trace.read_dataset(path, yname, dtype=np.float64)
        return X, y

    X_train, y_train = read("mnist_train.h5", "X_train", "y_train")
    X_test, y_test = read("mnist_test.h5", "X_test", "y_test")
    classes = np.unique(y_train)
    K = len(classes)
    y_train = one_hot(y_train[:], K)
    y_test = one_hot(y_test[:], K)
    if device is None:
        return X_train, y_train, X_test, y_test
    import torch
    dt = dtype or torch.float64
    return tuple(torch.as_tensor(a).to(device, dt).contiguous() for a in (X_train, y_train, X_test, y_test))
