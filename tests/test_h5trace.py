"""HDF5 trace backend (include/hmcx_trace.h, h5trace.py) on the CPU: the file layout of the
reference's multi-chain backend (cpu/sghmc_multicore.py:36-53 — float32 datasets (1,)+shape,
unlimited rows, zero first row) and backend_mean (cpu/hmc.py:132-138) against the oracle's
restatement.  The layout is also checked with the HDF5 distribution's own h5dump."""
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

from dropout_hamiltonian_montecarlo_amd import h5trace
from oracle import samplers as osm

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(not os.path.exists(h5trace._LIB_PATH), reason="libhmcx_trace.so not built")


def test_exports_match_header():
    hdr = open(os.path.join(REPO, "include", "hmcx_trace.h")).read()
    declared = set(re.findall(r"^\s*(?:int|int64_t|hmcx_trace\*|const char\*)\s+(hmcx_[a-z0-9_]+)\s*\(", hdr, re.M))
    assert declared == set(h5trace.EXPORTS)
    lib = h5trace.load_library()
    for sym in declared:
        assert hasattr(lib, sym), sym


def test_roundtrip_and_layout(tmp_path):
    D, K = 7, 3
    path = tmp_path / "backend_0.h5"
    rng = np.random.RandomState(0)
    wrows = [rng.standard_normal((n, D, K)) for n in (1, 5, 2)]
    brows = [rng.standard_normal((n, K)) for n in (1, 5, 2)]
    with h5trace.TraceFile(path, {"weights": (D, K), "bias": (K,)}) as f:
        assert f.rows("weights") == 1 and f.rows("bias") == 1
        for w, b in zip(wrows, brows):
            f.append("weights", w)
            f.append("bias", b)
            f.flush()
        assert f.rows("weights") == 9
    assert h5trace.list_datasets(path) == ["bias", "weights"]            # h5py keys(): name order
    W = h5trace.read_dataset(path, "weights")
    b = h5trace.read_dataset(path, "bias")
    assert W.dtype == np.float32 and W.shape == (9, D, K) and b.shape == (9, K)
    np.testing.assert_array_equal(W[0], 0.0)                              # the (1,)+shape fill row
    np.testing.assert_array_equal(W[1:], np.concatenate(wrows).astype(np.float32))
    np.testing.assert_array_equal(b[1:], np.concatenate(brows).astype(np.float32))
    h5dump = shutil.which("h5dump") or "/opt/conda/bin/h5dump"
    if os.path.exists(h5dump):
        out = subprocess.run([h5dump, "-H", str(path)], capture_output=True, text=True, check=True).stdout
        assert 'DATASET "weights"' in out and "H5T_IEEE_F32LE" in out
        assert "( 9, 7, 3 ) / ( H5S_UNLIMITED, 7, 3 )" in out
        assert "( 9, 3 ) / ( H5S_UNLIMITED, 3 )" in out


def test_backend_mean_matches_oracle(tmp_path):
    start = {"weights": np.zeros((4, 2)), "bias": np.zeros(2)}
    files, arrays = [], []
    for i in range(3):
        rng = np.random.RandomState(10 + i)
        p = str(tmp_path / ("b_%d.h5" % i))
        with h5trace.TraceFile(p, {"weights": (4, 2), "bias": (2,)}) as f:
            w, b = rng.standard_normal((6, 4, 2)), rng.standard_normal((6, 2))
            f.append("weights", w)
            f.append("bias", b)
        files.append(p)
        arrays.append({"bias": np.concatenate([np.zeros((1, 2)), b]).astype(np.float32),
                       "weights": np.concatenate([np.zeros((1, 4, 2)), w]).astype(np.float32)})
    got = h5trace.backend_mean(start, files, 18)
    want = osm.backend_mean_arrays(start, arrays, 18)
    for v in start:
        assert got[v].dtype == want[v].dtype
        np.testing.assert_array_equal(got[v], want[v])


def test_errors(tmp_path):
    with pytest.raises(h5trace.TraceError):
        h5trace.read_dataset(tmp_path / "missing.h5", "weights")
    p = tmp_path / "x.h5"
    with h5trace.TraceFile(p, {"w": (2,)}) as f:
        with pytest.raises(ValueError):
            f.append("w", np.zeros((3, 3)))                                # not a multiple of the row
    with pytest.raises(h5trace.TraceError):
        h5trace.read_dataset(p, "nope")


def test_mnist_loader(tmp_path):
    """benchmarks/2.-MNIST.ipynb cell 2 on synthetic MNIST-shaped files (uint8 images, int64
    labels): reshape to 784, /255., one_hot with K = #classes — identical to the notebook's
    NumPy expressions on the same arrays."""
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.data import load_mnist
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.utils import one_hot
    rng = np.random.RandomState(0)
    Xtr = rng.randint(0, 256, (50, 28, 28)).astype(np.uint8)
    ytr = rng.randint(0, 10, 50).astype(np.int64)
    Xte = rng.randint(0, 256, (20, 28, 28)).astype(np.uint8)
    yte = rng.randint(0, 10, 20).astype(np.int64)
    h5trace.write_dataset(tmp_path / "mnist_train.h5", "X_train", Xtr, truncate=True)
    h5trace.write_dataset(tmp_path / "mnist_train.h5", "y_train", ytr)
    h5trace.write_dataset(tmp_path / "mnist_test.h5", "X_test", Xte, truncate=True)
    h5trace.write_dataset(tmp_path / "mnist_test.h5", "y_test", yte)
    X_train, y_train, X_test, y_test = load_mnist(str(tmp_path))
    np.testing.assert_array_equal(X_train, Xtr.reshape((-1, 784)) / 255.)
    np.testing.assert_array_equal(X_test, Xte.reshape((-1, 784)) / 255.)
    K = len(np.unique(ytr))
    np.testing.assert_array_equal(y_train, one_hot(ytr, K))
    np.testing.assert_array_equal(y_test, one_hot(yte, K))
    assert h5trace.list_datasets(tmp_path / "mnist_train.h5") == ["X_train", "y_train"]
