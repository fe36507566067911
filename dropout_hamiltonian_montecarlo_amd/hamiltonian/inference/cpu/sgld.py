"""hamiltonian.inference.cpu.sgld — import path of /root/reference/hamiltonian/inference/cpu/sgld.py, served by
the libhmcx sampler of hamiltonian.inference.gpu.sgld (NumPy in / NumPy out, same signatures)."""
from ..gpu.sgld import sgld  # noqa: F401
