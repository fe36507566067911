"""sghmc_multicore — drop-in for hamiltonian/inference/cpu/sghmc_multicore.py:19-98.

``multicore_sample(X_train, y_train, niter, burnin, batch_size, backend, ncores)`` runs ncores
independent SGHMC chains in one libhmcx call per pass and stores every step's state (HDF5
backend files or in-memory rows); see multicore.py.  ``noise`` defaults to 'philox'
(independent chains).
"""
from .multicore import _default_philox, multicore_mixin
from .sghmc import sghmc


class sghmc_multicore(multicore_mixin, sghmc):

    def __init__(self, model, start_p, **kwargs):
        super().__init__(model, start_p, **_default_philox(kwargs))
