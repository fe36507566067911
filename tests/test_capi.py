"""CPU-side checks of the C ABI: the library loads, exports every symbol include/hmcx.h
declares, validates arguments without touching a device, and its host Philox generator is
well formed.  (No compute call is made: there is no GPU here.)"""
import ctypes
import os
import re

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def nat():
    from dropout_hamiltonian_montecarlo_amd import _native
    _native.load_library()
    return _native


def test_exports_match_header(nat):
    hdr = open(os.path.join(REPO, "include", "hmcx.h")).read()
    declared = set(re.findall(r"^(?:int|void|const char\*)\s+(hmcx_[a-z0-9_]+)\s*\(", hdr, re.M))
    assert declared == set(nat.EXPORTS)
    lib = nat.load_library()
    for sym in declared:
        assert hasattr(lib, sym), sym
    assert lib.hmcx_version() == 10000


def test_argument_validation_without_device(nat):
    lib = nat.load_library()
    # null context → EINVAL, no HIP call made
    assert lib.hmcx_softmax_grad(None, 1, None, None, 1, 1, 1, 1, None, None, 0.0, None, None) == -1
    assert lib.hmcx_sghmc_run(None, None) == -1
    assert lib.hmcx_mlp_hmc_leapfrog(None, None) == -1
    assert lib.hmcx_chain_diagnostics(None, 1, 4, 1, None, None, None, 0, None) == -1
    assert lib.hmcx_last_error(None) == b"null context"


_MIRRORS = [("SamplerArgs", "hmcx_sampler_args"), ("SgdArgs", "hmcx_sgd_args"), ("MvnArgs", "hmcx_hmc_mvn_args"),
            ("MlpParams", "hmcx_mlp_params"), ("MlpSghmcArgs", "hmcx_mlp_sghmc_args"), ("HmcArgs", "hmcx_hmc_args"),
            ("MlpLeapfrogArgs", "hmcx_mlp_leapfrog_args")]


def test_struct_layout_matches_header(nat, tmp_path):
    """Every field offset and the size of each ctypes mirror equal what gcc computes from
    include/hmcx.h (a layout drift would silently corrupt arguments)."""
    import shutil
    import subprocess
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "hmcx.h"', "int main(void) {"]
    for py, c in _MIRRORS:
        st = getattr(nat, py)
        lines.append('printf("%s sizeof %%zu\\n", sizeof(%s));' % (py, c))
        for f in st._fields_:
            lines.append('printf("%s %s %%zu\\n", offsetof(%s, %s));' % (py, f[0], c, f[0]))
    lines += ["return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run([cc, "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {}
    for line in out:
        if line:
            py, name, val = line.split()
            got[(py, name)] = int(val)
    for py, _ in _MIRRORS:
        st = getattr(nat, py)
        assert ctypes.sizeof(st) == got[(py, "sizeof")], py
        for f in st._fields_:
            assert getattr(st, f[0]).offset == got[(py, f[0])], (py, f[0])


def test_philox_host_generator(nat):
    u = nat.philox_uniforms(1234, 0, 7, 0, 20000)
    assert u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 0.01
    np.testing.assert_array_equal(u, nat.philox_uniforms(1234, 0, 7, 0, 20000))
    assert not np.array_equal(u, nat.philox_uniforms(1234, 1, 7, 0, 20000))   # chain key
    z = nat.philox_normals(99, 3, 1, 2, 0, 40000)
    assert abs(z.mean()) < 0.03 and abs(z.std() - 1) < 0.03
    # element ranges are position-addressed (counter-based): any split gives the same stream
    np.testing.assert_array_equal(z[101:205], nat.philox_normals(99, 3, 1, 2, 101, 104))


def test_philox_known_answer(nat):
    """Random123 Philox4x32-10 known-answer vector (counter = key = 0)."""
    lib = nat.load_library()
    # u53 of the first two output words of philox4x32_10({0,0,0,0}, {0,0}) = 0x6627e8d5, 0xe169c58d
    u = nat.philox_uniforms(0, 0, 0, 0, 1)[0]
    expect = ((0x6627e8d5 << 21) ^ (0xe169c58d >> 11)) / 2.0 ** 53
    assert u == expect


def test_philox_schedule_matches_vectorised_twin(nat):
    """hmcx_philox_schedule (one host C call per sampler call) equals the NumPy twin of the device
    generator, including the uint32 wrap of chain and step ids."""
    eps = np.array([1e-3, 5e-4, 1e-3, 2e-3, 1e-3])
    for seed, chain0, C, step0 in ((20251015, 0, 1, 0), (7, 0xFFFFFFFE, 3, 0xFFFFFFFD), (11, 64, 16, 1234567)):
        L, n_iter, u = nat.philox_schedule(seed, chain0, C, step0, 1e-2, eps)
        g = ((step0 + np.arange(len(eps))) & 0xFFFFFFFF)[:, None]
        ch = ((chain0 + np.arange(C)) & 0xFFFFFFFF)[None, :]
        uL = nat.philox_uniforms_chains(seed, ch, g, nat.SLOT_PATH)
        np.testing.assert_array_equal(L, np.ceil(2 * uL * 1e-2 / eps[:, None]))
        np.testing.assert_array_equal(n_iter, np.maximum(0, L - 1).astype(np.int32))
        np.testing.assert_array_equal(u, nat.philox_uniforms_chains(seed, ch, g, nat.SLOT_ACCEPT))
    with pytest.raises(nat.HmcxError):
        nat.philox_schedule(1, 0, 1, 0, 1e-2, np.array([0.0]))


def test_python_surface_imports():
    import hamiltonian.inference.gpu.sghmc as m1
    import hamiltonian.inference.gpu.sgld as m2
    import hamiltonian.inference.gpu.hmc as m3
    import hamiltonian.models.gpu.softmax as m4
    import hamiltonian.models.gpu.mvn_gaussian as m5
    import hamiltonian.models.gpu.logistic as m6
    import hamiltonian.inference.gpu.sgd as m7
    import hamiltonian.utils as u
    assert hasattr(m1, "sghmc") and hasattr(m2, "sgld") and hasattr(m3, "hmc")
    assert hasattr(m4, "softmax") and hasattr(m5, "mvn_gaussian")
    assert hasattr(m6, "logistic") and hasattr(m7, "sgd")
    np.testing.assert_array_equal(u.one_hot([2, 0], 3), [[0, 0, 1], [1, 0, 0]])


# Every module path the reference's own files import and that exists in the reference tree
# (benchmarks/1.-Simulated_data.ipynb cells 6, 8, 10; models/cpu/*.py import hamiltonian.models.model;
# inference/*/sgmcmc subclasses), plus the remaining sampler modules of inference/cpu.
_REFERENCE_PATHS = {
    "hamiltonian.models.cpu.logistic": "logistic", "hamiltonian.models.cpu.softmax": "softmax",
    "hamiltonian.models.cpu.mvn_gaussian": "mvn_gaussian", "hamiltonian.models.gpu.logistic": "logistic",
    "hamiltonian.models.gpu.softmax": "softmax", "hamiltonian.models.gpu.mlp": "mlp",
    "hamiltonian.models.gpu.mvn_gaussian": "mvn_gaussian", "hamiltonian.models.model": "model",
    "hamiltonian.inference.cpu.sgd": "sgd", "hamiltonian.inference.cpu.hmc": "hmc",
    "hamiltonian.inference.cpu.sgmcmc": "sgmcmc", "hamiltonian.inference.cpu.sghmc": "sghmc",
    "hamiltonian.inference.cpu.sgld": "sgld", "hamiltonian.inference.cpu.sghmc_multicore": "sghmc_multicore",
    "hamiltonian.inference.cpu.sgld_multicore": "sgld_multicore", "hamiltonian.inference.gpu.sgd": "sgd",
    "hamiltonian.inference.gpu.sgmcmc": "sgmcmc", "hamiltonian.inference.gpu.sgld_multicore": "sgld_multicore",
}


def test_reference_import_paths_resolve():
    """The reference harness's import paths resolve to the libhmcx-backed classes: inference.cpu.X is
    the same sampler class as inference.gpu.X, models.cpu.X a NumPy-surface subclass of models.gpu.X."""
    import importlib
    for path, name in _REFERENCE_PATHS.items():
        mod = importlib.import_module(path)
        assert hasattr(mod, name), path
    import hamiltonian.inference.cpu.hmc as hc
    import hamiltonian.inference.gpu.hmc as hg
    import hamiltonian.models.cpu.logistic as lc
    import hamiltonian.models.gpu.logistic as lg
    import hamiltonian.models.model as mm
    assert hc.hmc is hg.hmc and hasattr(hc, "DualAveragingStepSize")
    assert issubclass(lc.logistic, lg.logistic) and lc.logistic.__name__ == "logistic"
    assert lc.logistic._hmcx_model == "logistic"
    assert mm.model().grad(None, None) is None and mm.model().log_p(None, None) is None


def test_no_cpu_fallback():
    """The product fails loudly without a HIP device (no silent CPU path)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    from dropout_hamiltonian_montecarlo_amd._native import HmcxError
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.softmax import softmax
    with pytest.raises(HmcxError):
        softmax({"alpha": 0.01})
