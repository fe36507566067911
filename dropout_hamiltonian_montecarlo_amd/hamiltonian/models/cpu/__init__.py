"""hamiltonian.models.cpu — the reference's NumPy model import paths (models/cpu/*.py), served by the
libhmcx models with NumPy in / NumPy out (see _host.py)."""
