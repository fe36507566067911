"""hamiltonian.inference.cpu.sgd — import path of /root/reference/hamiltonian/inference/cpu/sgd.py, served by
the libhmcx sampler of hamiltonian.inference.gpu.sgd (NumPy in / NumPy out, same signatures)."""
from ..gpu.sgd import sgd  # noqa: F401
