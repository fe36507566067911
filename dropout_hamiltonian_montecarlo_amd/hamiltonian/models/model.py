"""hamiltonian.models.model — the model protocol of the reference (hamiltonian/models/model.py:1-7).

The reference's base class declares two hooks and nothing else; its samplers duck-type the rest
(grad / log_likelihood / negative_log_posterior).  The libhmcx-backed models
(hamiltonian.models.{cpu,gpu}.*) implement that surface; this class is kept so code written against
the protocol (``import hamiltonian.models.model as base_model``) imports unchanged.
"""


class model:
    """Protocol: ``log_p(par, hyper, *args)`` and ``grad(par, hyper, *args)``; both are no-ops here,
    exactly as in the reference (subclasses override them)."""

    def log_p(self, par, hyper, *args):
        return None

    def grad(self, par, hyper, *args):
        return None
