"""Loci-streamed fits on the GPU (csrc/capi.cpp stream_grm_shard / stream_effects_shard): a shard whose
fp64 locus rows do not fit HBM keeps its genotypes as int8 dosages (or on the host, fp64 input) and
passes the loci through one fp64 chunk buffer, each chunk's GRM added into G in place. That is how
config C3 (n = 50 000 x p = 600 000, BASELINE configs[2]) runs on one MI355X
(test_gpu_large.py::test_c3_full_size_one_gpu_streamed); here the mode is forced on small shapes
(GBM_STREAM_CHUNK) and checked against

* the oracle (GEBVs 1e-9, b_hat 1e-6 of max|b|; reference equations src/gwas.jl:462-472,591-597,
  src/prediction.jl:228),
* the resident path on the same input (rounding only: the chunk GRMs are summed in another order),
* the pipelined host upload over the same chunks (GBM_HOST_CHUNK): the same chunk GRMs summed in the
  same order, so the results are the SAME BITS, for int8 and fp64 input,
* the streamed stage path of gbm.sharded (HipStreamedShardStages), the one the C3 bench runs.
"""
import numpy as np
import pytest

import gbm
import oracle
from gbm import synth

pytestmark = pytest.mark.gpu

N, P, CHUNK, SEED = 700, 5000, 1500, 77


def rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(np.abs(np.asarray(b)).max(), 1e-300))


@pytest.fixture(scope="module")
def data():
    X = oracle.synth_genotypes(SEED, N, P)
    Y = oracle.synth_phenotypes(X, SEED + 1, ntraits=2)
    return X, Y


def _fit_synth(gbm_env, stream, Y, devices=(0,), host_chunk=None):
    gbm_env.setenv("GBM_STREAM_CHUNK", str(stream))
    if host_chunk:
        gbm_env.setenv("GBM_HOST_CHUNK", str(host_chunk))
    else:
        gbm_env.delenv("GBM_HOST_CHUNK", raising=False)
    return gbm.gblup_synthetic(SEED, N, P, Y, lambda_=1.0, devices=list(devices))


def test_streamed_synthetic_matches_oracle_and_resident(gbm_env, data):
    X, Y = data
    b, y, mu, q = _fit_synth(gbm_env, CHUNK, Y)
    ref = oracle.gblup_fit(X, Y, 1.0)
    assert q == ref["q"]
    assert rel(y, ref["y_pred"]) < 1e-9 and rel(mu, ref["mu"]) < 1e-9 and rel(b, ref["b_hat"]) < 1e-6
    b0, y0, mu0, q0 = _fit_synth(gbm_env, 0, Y)
    assert q0 == q and rel(y, y0) < 1e-12 and rel(b, b0) < 1e-10
    # the predict identity of reference src/prediction.jl:228 on the streamed fit
    assert rel(b[0] + X @ b[1:], y) < 1e-9


@pytest.mark.parametrize("host_chunk", [CHUNK, 1024])
def test_streamed_int8_same_bits_as_pipelined_upload(gbm_env, data, host_chunk):
    X, Y = data
    D = np.asfortranarray(np.rint(2.0 * X).astype(np.int8))
    gbm_env.setenv("GBM_HOST_CHUNK", str(host_chunk))
    gbm_env.setenv("GBM_STREAM_CHUNK", str(host_chunk))
    s = gbm.gblup_dosage(D, 2, Y)
    gbm_env.setenv("GBM_STREAM_CHUNK", "0")
    r = gbm.gblup_dosage(D, 2, Y)
    for a, b in zip(s, r):
        assert np.array_equal(np.asarray(a), np.asarray(b))


def test_streamed_fp64_same_bits_as_pipelined_and_int8(gbm_env, data):
    X, Y = data
    D = np.asfortranarray(np.rint(2.0 * X).astype(np.int8))
    gbm_env.setenv("GBM_HOST_CHUNK", str(CHUNK))
    gbm_env.setenv("GBM_STREAM_CHUNK", str(CHUNK))
    s = gbm.gblup_arrays(X, Y)
    s8 = gbm.gblup_dosage(D, 2, Y)
    gbm_env.setenv("GBM_STREAM_CHUNK", "0")
    r = gbm.gblup_arrays(X, Y)
    for a, b, c in zip(s, r, s8):
        assert np.array_equal(np.asarray(a), np.asarray(b))
        assert np.array_equal(np.asarray(a), np.asarray(c))


def test_streamed_synthetic_same_bits_as_streamed_int8(gbm_env, data):
    """On-device dosage generation == the same bytes uploaded from the host."""
    X, Y = data
    D = np.asfortranarray(np.rint(2.0 * X).astype(np.int8))
    s = _fit_synth(gbm_env, CHUNK, Y)
    r = gbm.gblup_dosage(D, 2, Y)  # GBM_STREAM_CHUNK still set by _fit_synth
    for a, b in zip(s, r):
        assert np.array_equal(np.asarray(a), np.asarray(b))


def test_streamed_single_range_tail_chunk(gbm_env, data):
    """A last chunk too small for a multi-range GRM plan goes through its own G and an add (Gc)."""
    X, Y = data
    lib = gbm.load_library()
    chunk = P - 16  # tail of 16 loci
    assert lib.gbm_dev_grm_slices(N, 16) == 1 and lib.gbm_dev_grm_slices(N, chunk) > 1
    b, y, mu, q = _fit_synth(gbm_env, chunk, Y)
    b0, y0, mu0, q0 = _fit_synth(gbm_env, 0, Y)
    assert q == q0 and rel(y, y0) < 1e-12 and rel(b, b0) < 1e-10


def test_streamed_two_shards_one_device(gbm_env, data):
    X, Y = data
    b, y, mu, q = _fit_synth(gbm_env, 1000, Y, devices=(0, 0))
    b0, y0, mu0, q0 = _fit_synth(gbm_env, 0, Y, devices=(0, 0))
    assert q == q0 and rel(y, y0) < 1e-12 and rel(b, b0) < 1e-10


def test_streamed_reml(gbm_env, data):
    X, Y = data
    gbm_env.setenv("GBM_STREAM_CHUNK", str(CHUNK))
    s = gbm.gblup_reml_arrays(X, Y)
    gbm_env.setenv("GBM_STREAM_CHUNK", "0")
    r = gbm.gblup_reml_arrays(X, Y)
    assert rel(s[1], r[1]) < 1e-9 and rel(s[4]["lambda"], r[4]["lambda"]) < 1e-8


def test_streamed_stage_path_matches_c_abi(gbm_env, data):
    import torch
    from gbm.sharded import HipStreamedShardStages, assemble_b_hat

    X, Y = data
    st = HipStreamedShardStages(N, P, CHUNK, nrhs=2, lambda_=1.0, device=0)
    st.generate(SEED, 0)
    st.load_phenotypes(Y)
    st.standardize()
    st.grm_syrk()
    st.grm_reduce()
    st.solve()
    st.effects()
    out = st.download()
    q = int(st.q.item())
    b_st = assemble_b_hat(out["mu"], out["msum"], [out["B"]], P)
    del st
    torch.cuda.empty_cache()
    b, y, mu, q2 = _fit_synth(gbm_env, CHUNK, Y)
    assert q == q2
    assert rel(out["y_pred"], y) < 1e-13 and rel(b_st, b) < 1e-12


def test_grm_accumulate_rejects_single_range_plan():
    import ctypes

    import torch
    lib = gbm.load_library()
    n, p = 300, 16
    assert lib.gbm_dev_grm_slices(n, p) == 1
    npad, gdim = lib.gbm_dev_npad(n), lib.gbm_dev_gdim(n)
    Z = torch.zeros((p, npad), dtype=torch.float64, device="cuda")
    G = torch.zeros((gdim, gdim), dtype=torch.float64, device="cuda")
    ws = torch.empty(max(lib.gbm_dev_grm_workspace(n, p), 16), dtype=torch.uint8, device="cuda")
    rc = lib.gbm_dev_grm_accumulate(ctypes.c_void_p(Z.data_ptr()), npad, p, n, ctypes.c_void_p(G.data_ptr()), gdim,
                                    ctypes.c_void_p(ws.data_ptr()), ws.numel(), None)
    assert rc == gbm._lib.GBM_E_ARG
