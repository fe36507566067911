"""hamiltonian/utils.py (reference utils.py:1-26) for Python ≥ 3.10 / NumPy 2."""
from collections.abc import Iterable

import numpy as np


def one_hot(y, num_classes):
    """utils.py:4-8 — float64 [N, K] label matrix the softmax model consumes."""
    y = np.asarray(y)
    encoding = np.zeros((len(y), num_classes))
    encoding[np.arange(len(y)), y.astype(int)] = 1.0
    return encoding


def scaler_fit(X):
    """utils.py:10-14."""
    min_col = np.amin(X, 0)
    max_col = np.amax(X, 0)
    X_s = (X - min_col) / (max_col - min_col)
    return X_s, min_col, max_col


def scaler_scale(X, min_col, max_col):
    """utils.py:16-18."""
    return (X - min_col) / (max_col - min_col)


def flatten(items):
    """utils.py:20-26."""
    for x in items:
        if isinstance(x, Iterable) and not isinstance(x, (str, bytes)):
            for sub_x in flatten(x):
                yield sub_x
        else:
            yield x
