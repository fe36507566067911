"""hamiltonian.inference.cpu.sghmc — import path of /root/reference/hamiltonian/inference/cpu/sghmc.py, served by
the libhmcx sampler of hamiltonian.inference.gpu.sghmc (NumPy in / NumPy out, same signatures)."""
from ..gpu.sghmc import sghmc  # noqa: F401
