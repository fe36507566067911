"""hamiltonian.models.cpu.softmax — import path of the reference's /root/reference/hamiltonian/models/cpu/softmax.py
(the reference's NumPy model): NumPy in / NumPy out, computed by the libhmcx model
hamiltonian.models.gpu.softmax."""
from ..gpu.softmax import softmax as _device_softmax
from ._host import host_surface

softmax = host_surface(_device_softmax)
