"""hamiltonian.inference.cpu — the reference's NumPy sampler import paths (inference/cpu/*.py).

The libhmcx samplers already take NumPy inputs and return NumPy results with the reference's
signatures, so each module here names the same class as its inference.gpu twin: one implementation,
both import paths (benchmarks/1.-Simulated_data.ipynb imports inference.cpu.sgd and inference.cpu.hmc).
"""
