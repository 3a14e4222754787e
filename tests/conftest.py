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
