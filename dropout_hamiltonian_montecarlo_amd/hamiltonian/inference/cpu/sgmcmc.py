"""hamiltonian.inference.cpu.sgmcmc — import path of /root/reference/hamiltonian/inference/cpu/sgmcmc.py, served by
the libhmcx sampler of hamiltonian.inference.gpu.sgmcmc (NumPy in / NumPy out, same signatures)."""
from ..gpu.sgmcmc import sgmcmc  # noqa: F401
