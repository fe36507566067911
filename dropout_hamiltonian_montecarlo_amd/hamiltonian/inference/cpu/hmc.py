"""hamiltonian.inference.cpu.hmc — import path of /root/reference/hamiltonian/inference/cpu/hmc.py, served by
the libhmcx sampler of hamiltonian.inference.gpu.hmc (NumPy in / NumPy out, same signatures)."""
from ..gpu.hmc import hmc, DualAveragingStepSize  # noqa: F401
