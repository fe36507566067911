"""MI355X-native stochastic-gradient HMC engine (drop-in for sherna90/dropout_hamiltonian_montecarlo's
leapfrog + minibatch-gradient hot path).

Layout:
  csrc/        hand-written HIP kernels for gfx950 + the C ABI (include/hmcx.h) → lib/libhmcx.so
  _native.py   ctypes binding (fails loudly when the library or a HIP device is missing)
  hamiltonian/ host-side mirror of the reference's Python surface:
               hamiltonian.models.gpu.{softmax,mlp,mvn_gaussian}, hamiltonian.inference.gpu.{sghmc,sgld,hmc}
  parallel.py  one-process-per-GPU chain sharding + RCCL gather of chain statistics (R-hat / ESS)
"""
__version__ = "0.1.0"
