"""sgld_multicore — drop-in for hamiltonian/inference/gpu/sgld_multicore.py:19-90.

``multicore_sample(X_train, y_train, niter, burnin, batch_size, backend, ncores)`` runs ncores
independent SGLD chains in one libhmcx call per pass and stores every step's state (HDF5
backend files or in-memory rows); see multicore.py.  ``noise`` defaults to 'philox'
(independent chains); ``variant='gpu'`` selects the CuPy file's momentum update.
"""
from .multicore import _default_philox, multicore_mixin
from .sgld import sgld


class sgld_multicore(multicore_mixin, sgld):

    def __init__(self, model, start_p, **kwargs):
        super().__init__(model, start_p, **_default_philox(kwargs))
