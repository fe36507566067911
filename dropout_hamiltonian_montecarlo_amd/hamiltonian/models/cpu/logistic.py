"""hamiltonian.models.cpu.logistic — import path of the reference's /root/reference/hamiltonian/models/cpu/logistic.py
(imported by benchmarks/1.-Simulated_data.ipynb cell 6): NumPy in / NumPy out, computed by the libhmcx model
hamiltonian.models.gpu.logistic."""
from ..gpu.logistic import logistic as _device_logistic
from ._host import host_surface

logistic = host_surface(_device_logistic)
