"""CPU tests of the C-ABI boundary: libgbm.so loads, exports every symbol include/gbm.h declares,
reports its version, and fails loudly (never silently falls back) when no GPU is present."""
import os
import re
import subprocess

import numpy as np
import pytest

import gbm
from gbm import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gbm.h")


def header_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gbm_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_bound_symbols():
    assert header_symbols() == sorted(_lib.EXPORTS)


def test_library_exports_every_header_symbol():
    assert os.path.exists(_lib.LIB_PATH), "build first: __graft_entry__.build()"
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    exported = set(re.findall(r" T (gbm_[a-z0-9_]+)", out))
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing


def test_library_loads_and_reports_version():
    lib = gbm.load_library()
    assert lib.gbm_version() == 200
    assert isinstance(_lib.last_error(), str)
    for s in _lib.EXPORTS:
        assert hasattr(lib, s)


def test_geometry_helpers():
    lib = gbm.load_library()
    assert lib.gbm_dev_npad(1) == 128 and lib.gbm_dev_npad(5000) == 5120 and lib.gbm_dev_npad(5120) == 5120
    assert lib.gbm_dev_gdim(5000) == 5120 + 64
    # Ld, Linv, Dinv, back-substitution flags; then (16-byte aligned) the dataflow queue + tile flags
    nbc = (5120 + 64) // 64
    assert lib.gbm_dev_solve_workspace(5000, 1) == (5120 * (2 * 64 + 16) + 40 + 1 + 1) * 8 + (16 + nbc * nbc * 4 + 15) // 16 * 16
    # GRM workspace: loci-slice partial tiles (+ the ragged-column partials when n % 128 <= 64)
    # (+ 32 bytes of queue counters for the persistent launch)
    assert (lib.gbm_dev_grm_workspace(5120, 50000) - 32) % (128 * 128 * 8) == 0
    assert lib.gbm_dev_grm_workspace(5000, 50000) > 0


def test_no_gpu_means_loud_error():
    if gbm.device_count() > 0:
        pytest.skip("a GPU is visible; covered by the -m gpu tests")
    X = np.random.default_rng(0).random((20, 30))
    with pytest.raises(gbm.GBMError, match="no HIP device"):
        gbm.gblup_arrays(X, np.arange(20.0))
    with pytest.raises(gbm.GBMError):
        gbm.grm(X)


def test_argument_errors_before_device_use():
    X = np.random.default_rng(0).random((20, 30))
    with pytest.raises(gbm.ArgumentError):
        gbm.gblup_arrays(X, np.arange(20.0), lambda_=-1.0)
    with pytest.raises(gbm.ArgumentError):
        gbm.gblup_arrays(X, np.r_[np.arange(19.0), np.nan])
    with pytest.raises(gbm.GBMError, match="variance"):
        gbm.gblup_arrays(X, np.ones(20))
    with pytest.raises(gbm.GBMError, match="less than 2"):
        gbm.gblup_arrays(X[:1], np.ones(1))
