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
    assert lib.gbm_version() == 212
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


def test_distributed_phase_entry_points_check_their_arguments():
    """The distributed-factorisation phases (include/gbm.h) refuse a bad step, rank or range before
    any device work (fake, aligned pointers: nothing is dereferenced on the host)."""
    import ctypes
    lib = gbm.load_library()
    n = 3000
    G = ctypes.c_void_p(1 << 20)  # 16-byte aligned, never touched
    ws_bytes = lib.gbm_dev_solve_workspace(n, 1)
    ws, info = ctypes.c_void_p(1 << 21), ctypes.c_void_p(1 << 22)
    gdim = lib.gbm_dev_gdim(n)
    E = _lib.GBM_E_ARG
    # gbm_dev_chol_group is the one-rank step only
    assert lib.gbm_dev_chol_group(G, gdim, n, 0, 1, 2, info, ws, ws_bytes, None) == E
    assert "one rank only" in _lib.last_error()
    # the column-range update needs nranks >= 2 and an ordered range
    assert lib.gbm_dev_chol_group_update_cols(G, gdim, n, 0, 0, 1, 0, gdim, info, ws, ws_bytes, None) == E
    assert lib.gbm_dev_chol_group_update_cols(G, gdim, n, 0, 0, 2, 512, 256, info, ws, ws_bytes, None) == E
    assert lib.gbm_dev_chol_group_update_tiles(G, gdim, n, 0, 0, 1, 0, gdim, 0, gdim, info, ws, ws_bytes, None) == E
    assert lib.gbm_dev_chol_prepare_cols(G, gdim, n, 1.0, None, 1.0, G, n, 1, 2, 2, info, ws, ws_bytes, None) == E
    assert lib.gbm_dev_chol_group_update_tiles(G, gdim, n, 0, 0, 2, 256, 128, 0, gdim, info, ws, ws_bytes, None) == E
    # a rank outside [0, nranks)
    assert lib.gbm_dev_chol_group_panels(G, gdim, n, 0, 2, 2, info, ws, ws_bytes, None) == E
    assert lib.gbm_dev_chol_group_update(G, gdim, n, 0, -1, 2, info, ws, ws_bytes, None) == E
    # a distributed panel phase on a single-panel step (the last block)
    nb = lib.gbm_dev_npad(n) // 64
    assert lib.gbm_dev_chol_group_size(n, nb - 1) == 1
    assert lib.gbm_dev_chol_group_panels(G, gdim, n, nb - 1, 0, 2, info, ws, ws_bytes, None) == E
    # the area exchange covers a square ending on a 128-row boundary
    assert lib.gbm_dev_chol_area_pack(G, gdim, n, 0, 3, 0, 2, ctypes.c_void_p(1 << 23), None) == E
    assert lib.gbm_dev_chol_area_doubles(n, 0, 4, 2) == 1 * 256 * 128  # ⌈2 tiles / 2 ranks⌉ x 256 rows x 128
    assert lib.gbm_dev_chol_strip_unpack_rows(G, gdim, n, 0, 2, 3, 2, ctypes.c_void_p(1 << 23), None) == E


def test_grm_mode_is_checked_before_device_use():
    """grm_mode (include/gbm.h GBM_GRM_*) is a per-call argument: an unknown mode, or exact on int8 dosages of
    another ploidy, is an argument error before any device work; the Python mirror maps names to modes."""
    X = np.asfortranarray(np.random.default_rng(0).random((20, 30)))
    y = np.arange(20.0)
    b, yp = np.zeros(31), np.zeros(20)
    lib = gbm.load_library()
    assert lib.gbm_gblup_fit_ex(_lib.ptr(X), 20, 30, 20, _lib.ptr(y), 20, 1, 1.0, None, 0, 7, _lib.ptr(b),
                                _lib.ptr(yp), None, None, None) == _lib.GBM_E_ARG
    assert "grm_mode" in _lib.last_error()
    with pytest.raises(gbm.ArgumentError, match="grm must be"):
        gbm.gblup_arrays(X, np.arange(20.0), grm="int8")
    D = np.random.default_rng(1).integers(0, 5, (20, 30)).astype(np.int8)
    with pytest.raises(gbm.ArgumentError, match="ploidy 2"):
        gbm.gblup_dosage(D, 4, np.arange(20.0), grm="exact")
    assert _lib.grm_mode(None) == -1 and _lib.grm_mode("auto") == 2 and _lib.grm_mode("exact") == 1


def test_rccl_call_counters_start_at_zero():
    import ctypes
    a, g = ctypes.c_int64(-1), ctypes.c_int64(-1)
    assert gbm.load_library().gbm_debug_rccl_calls(ctypes.byref(a), ctypes.byref(g)) == 0
    assert a.value >= 0 and g.value >= 0


def _order_tiles(buf):
    """Decode a dequeue order: (i, j) per tile, a pair entry (bit 15) giving (i, j) and (i, j + 1) at one position."""
    out = []
    for t, v in enumerate(buf):
        i, j = v >> 16, v & 0x7FFF
        out += [(t, i, j)] + ([(t, i, j + 1)] if v & 0x8000 else [])
    return out


@pytest.mark.parametrize("variant", ["default", "6", "4"])
def test_chol_flow_dequeue_order_is_complete_and_deadlock_free(gbm_env, variant):
    """The dataflow Cholesky's worker dequeue order (csrc/chol_flow.hip flow_order, host-built): every upper
    64-tile except (0, 0) once, each task after everything it waits for (k-loop operands and the chain's inputs),
    checked on the host for every tile count the dataflow path runs (npad <= 12 288: nbc <= 193); the diagonal
    partial (d, d) follows (d − 2, d) directly (two rows early); the tiles (r, j >= r + 3) go in pairs (one k-loop
    for two tiles), the tiles the chain and the assistant wait for alone."""
    import ctypes
    if variant != "default":  # GBM_CHOL_FLOW_ORDER is read at every call
        gbm_env.setenv("GBM_CHOL_FLOW_ORDER", variant)
    pairs = variant == "6"
    lib = gbm.load_library()
    for nbc in range(2, 194):
        m = lib.gbm_debug_chol_flow_order_size(nbc)
        buf = (ctypes.c_int32 * m)()
        assert lib.gbm_debug_chol_flow_order(nbc, buf, m) == 0, nbc
        tiles = _order_tiles(buf)
        assert len(tiles) == nbc * (nbc + 1) // 2 - 1
        assert len({(i, j) for _, i, j in tiles}) == len(tiles)
        pos = {(i, j): t for t, i, j in tiles}
        if variant != "4":
            for d in range(2, nbc - 2):
                assert pos[(d, d)] == pos[(d - 2, d)] + 1
        for t, v in enumerate(buf):
            i, j = v >> 16, v & 0x7FFF
            if v & 0x8000:
                assert pairs and j >= i + 3 and j + 1 <= nbc - 1
            elif j >= i + 3 and pairs:
                assert j == nbc - 1  # a row's odd last tile
        assert (m < nbc * (nbc + 1) // 2 - 1) == (pairs and nbc >= 5)
    assert lib.gbm_debug_chol_flow_order(1, None, 0) == -1
    assert lib.gbm_debug_chol_flow_order_size(1) == -1
    # the checker itself: a diagonal partial moved in front of its last operand, a tile in front of the chain's
    # input of its row, a missing entry, a duplicated tile and a pair over a chain input are caught; plain
    # row-major order with the partials first and no pairs is valid
    if variant == "4":  # (the swaps below are placed for the two-rows-early diagonal partials)
        gbm_env.delenv("GBM_CHOL_FLOW_ORDER")
    nbc = 20
    m = lib.gbm_debug_chol_flow_order_size(nbc)
    buf = (ctypes.c_int32 * m)()
    lib.gbm_debug_chol_flow_order(nbc, buf, m)
    order = list(buf)

    def check(o):
        arr = (ctypes.c_int32 * len(o))(*o)
        return lib.gbm_debug_chol_flow_order_check(nbc, arr, len(o))

    assert check(order) == 0
    enc = lambda i, j: (i << 16) | j
    bad = order.copy()
    t = bad.index(enc(7, 7))
    bad[t], bad[t - 1] = bad[t - 1], bad[t]  # (7, 7) before (5, 7)
    assert check(bad) == t
    bad = order.copy()
    a, b = bad.index(enc(6, 7)), bad.index(enc(6, 8))  # the chain's step-6 input after a tile waiting for step 6
    bad[a], bad[b] = bad[b], bad[a]
    assert check(bad) != 0
    assert check(order[:-1]) != 0
    if pairs:
        bad = order.copy()
        p = next(t for t, v in enumerate(bad) if v & 0x8000)
        bad[p] &= 0x7FFF7FFF  # a pair entry split: its second tile is missing
        assert check(bad) != 0
    assert check(order + [enc(5, 9)]) != 0
    assert check([enc(0, 1) | 0x8000] + order[1:]) != 0
    rowmajor = [enc(0, 1), enc(1, 1)]
    for r in range(nbc):
        if r >= 1 and r + 1 <= nbc - 1:
            rowmajor += [enc(r, r + 1)] + ([enc(r + 1, r + 1)] if r + 1 < nbc - 1 else [])
        rowmajor += [enc(r, j) for j in range(r + 2, nbc)]
    rowmajor.append(enc(nbc - 1, nbc - 1))
    assert check(rowmajor) == 0
