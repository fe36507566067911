"""ORACLE — test infrastructure only, never the product.

CPU restatement (NumPy, float64) of the reference's hot path:
``hamiltonian.models.cpu.softmax``, ``hamiltonian.models.cpu.mvn_gaussian``,
``hamiltonian.models.gpu.mlp`` (restated in NumPy with injected dropout masks),
and the samplers ``hamiltonian.inference.cpu.{sgmcmc,sghmc,sgld,hmc}``.
Every function cites the reference ``file:line`` it follows.

Who may import this package: ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` — as the CHECKER only.  The product
(``dropout_hamiltonian_montecarlo_amd``) never imports it and fails loudly when
its HIP library is missing.

Pinning: ``oracle/gen_golden.py`` (run in the build container, where the
reference is importable through a small import shim) executes the reference's
own code and writes ``tests/golden/*.npz``; ``tests/test_oracle_golden.py``
checks this restatement against those vectors bit-for-bit.  The MLP restatement
has no runnable reference (Chainer/CuPy absent): *parity unpinned*, cross-checked
against PyTorch CPU autograd instead.
"""
