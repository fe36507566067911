"""hamiltonian.inference.cpu.sghmc_multicore — import path of /root/reference/hamiltonian/inference/cpu/sghmc_multicore.py, served by
the libhmcx sampler of hamiltonian.inference.gpu.sghmc_multicore (NumPy in / NumPy out, same signatures)."""
from ..gpu.sghmc_multicore import sghmc_multicore  # noqa: F401
