import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "genomicbreedingmodels.jl_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: larger sizes")


@pytest.fixture(scope="session")
def oracle_c():
    """ctypes handle of the C restatement (oracle/build/libgbm_oracle.so), built on demand."""
    import ctypes
    import subprocess
    so = os.path.join(ROOT, "oracle", "build", "libgbm_oracle.so")
    if not os.path.exists(so):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    lib = ctypes.CDLL(so)
    P, I, D, U = ctypes.c_void_p, ctypes.c_int64, ctypes.c_double, ctypes.c_uint64
    lib.gbm_ref_synth_genotype.restype = D
    lib.gbm_ref_synth_genotype.argtypes = [U, I, I]
    lib.gbm_ref_synth_matrix.restype = None
    lib.gbm_ref_synth_matrix.argtypes = [U, I, I, I, P, I]
    lib.gbm_ref_colstats.restype = I
    lib.gbm_ref_colstats.argtypes = [P, I, I, I, P, P, P]
    lib.gbm_ref_grm.restype = I
    lib.gbm_ref_grm.argtypes = [P, I, I, I, P, I]
    lib.gbm_ref_gblup_fit.restype = I
    lib.gbm_ref_gblup_fit.argtypes = [P, I, I, I, P, I, I, D, P, P, P, P]
    return lib


class _GbmEnv:
    """monkeypatch.setenv / delenv for GBM_* knobs: libgbm reads its environment once (csrc/knobs.cpp), so a
    knob a test changes goes through gbm_debug_set (gbm._lib.debug_set, which also updates os.environ for the
    Python-level knobs); every knob touched is restored when the test ends."""

    def __init__(self):
        self._saved = {}

    def _save(self, name):
        if name not in self._saved:
            self._saved[name] = os.environ.get(name)

    def setenv(self, name, value):
        from gbm import _lib
        self._save(name)
        _lib.debug_set(name, str(value))

    def delenv(self, name, raising=True):
        from gbm import _lib
        if raising and name not in os.environ:
            raise KeyError(name)
        self._save(name)
        _lib.debug_set(name, None)

    def undo(self):
        from gbm import _lib
        for name, value in self._saved.items():
            _lib.debug_set(name, value)
        self._saved.clear()


@pytest.fixture
def gbm_env():
    env = _GbmEnv()
    yield env
    env.undo()
