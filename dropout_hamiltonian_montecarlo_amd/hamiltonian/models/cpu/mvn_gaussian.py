"""hamiltonian.models.cpu.mvn_gaussian — import path of the reference's /root/reference/hamiltonian/models/cpu/mvn_gaussian.py
(the reference's NumPy model): NumPy in / NumPy out, computed by the libhmcx model
hamiltonian.models.gpu.mvn_gaussian."""
from ..gpu.mvn_gaussian import mvn_gaussian as _device_mvn_gaussian
from ._host import host_surface

mvn_gaussian = host_surface(_device_mvn_gaussian)
