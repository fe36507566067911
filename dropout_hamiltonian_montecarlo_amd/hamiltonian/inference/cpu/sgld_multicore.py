"""hamiltonian.inference.cpu.sgld_multicore — import path of /root/reference/hamiltonian/inference/cpu/sgld_multicore.py, served by
the libhmcx sampler of hamiltonian.inference.gpu.sgld_multicore (NumPy in / NumPy out, same signatures)."""
from ..gpu.sgld_multicore import sgld_multicore  # noqa: F401
