"""Host-array surface shared by hamiltonian.models.cpu.*.

The reference's CPU models (models/cpu/{softmax,logistic,mvn_gaussian}.py) take and return NumPy
arrays; the libhmcx models return device tensors.  ``host_surface(cls)`` derives a class whose
``grad`` / ``net`` hand back NumPy arrays (a device→host copy of the kernel results) while every
computation still runs in libhmcx; the samplers (which call the fused entries, not ``grad``) use
the class unchanged.
"""
import numpy as np
import torch


def _host(v):
    return v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)


def host_surface(base):
    class cls(base):
        __doc__ = ("NumPy-in / NumPy-out surface of the reference's CPU model, computed by libhmcx "
                   "(%s.%s)." % (base.__module__, base.__name__))

        def grad(self, par, **args):
            return {k: _host(v) for k, v in base.grad(self, par, **args).items()}

        if hasattr(base, 'net'):
            def net(self, *a, **kw):
                return _host(base.net(self, *a, **kw))

    cls.__name__ = cls.__qualname__ = base.__name__
    return cls
