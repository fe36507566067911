"""Drop-in alias for the reference's import paths.

``import hamiltonian.inference.gpu.sghmc`` / ``hamiltonian.models.gpu.softmax`` (the module
paths of /root/reference/hamiltonian) resolve to the libhmcx-backed implementation in
dropout_hamiltonian_montecarlo_amd/hamiltonian, so the reference's benchmark scripts run
unchanged with this repository on sys.path.
"""
import dropout_hamiltonian_montecarlo_amd.hamiltonian as _impl

__path__ = _impl.__path__
