"""The HIP path pinned to the committed golden fixtures and to the reference's own doctest
properties, and the GRM accumulation modes forced per call.

* tests/golden/*.npz (tests/golden/make_golden.py): int8 dosage + ploidy, phenotypes (with
  missing values), λ, and the expected q, μ̂, GEBVs, b_hat, column stats and GRM entries. They go
  straight into the C ABI entries (gbm_gblup_fit_dosage_i8, gbm_gblup_fit, gbm_grm) and through
  the model function (whose extractxyetc drops the missing phenotypes, src/prediction.jl:114-131).
* gwasprep's doctest (src/gwas.jl:53-74): standardised columns have mean 0 and std 1 within
  1e-10, and size(GRM) == (n, n) — asserted on the HIP outputs.
* predict's doctest (src/prediction.jl:175-186): 100 entries, fit on 1:90, predict 91:100,
  cor > 0.5 — on a seeded related population of that shape.
* GBM_GRM_CARRY / GBM_GRM_PERSIST / GBM_GRM_SPLIT are read at every plan, so the in-order carry
  accumulation (the large-n mode) and the hardware-dispatched launch run on small ragged shapes.
"""
import ctypes
import glob
import json
import os

import numpy as np
import pytest

import gbm
import oracle
from gbm import _lib

pytestmark = pytest.mark.gpu

GOLD = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "*_*x*.npz")))
TOL_TIGHT = 1e-9
TOL_CONTRACT = 1e-6


def rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(np.abs(np.asarray(b)).max(), 1e-300))


def _fixture(path):
    z = np.load(path)  # plain arrays only (allow_pickle=False)
    keep = z["keep_rows"]
    D = np.asfortranarray(z["dosage"][keep])
    ploidy = int(z["ploidy"])
    Y = np.asfortranarray(z["phenotypes"][keep])
    return z, D, ploidy, Y


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_golden_fixture_dosage_and_host_entries(path):
    z, D, ploidy, Y = _fixture(path)
    n, p = D.shape
    t = Y.shape[1]
    lam = float(z["lam"])
    lib = gbm.load_library()
    b_hat = np.zeros((p + 1, t), order="F")
    y_pred = np.zeros((n, t), order="F")
    mu = np.zeros(t)
    q = np.zeros(1, dtype=np.int64)
    rc = lib.gbm_gblup_fit_dosage_i8(_lib.ptr(D), n, p, n, ploidy, _lib.ptr(Y), n, t, lam, None, 0,
                                     _lib.ptr(b_hat), _lib.ptr(y_pred), _lib.ptr(mu), _lib.ptr(q))
    _lib.check(rc, "gbm_gblup_fit_dosage_i8")
    assert q[0] == int(z["q"])
    assert rel(y_pred, z["y_pred"]) < TOL_TIGHT
    assert rel(mu, z["mu"]) < TOL_TIGHT
    assert rel(b_hat, z["b_hat"]) < TOL_CONTRACT
    # the fp64 host entry on X = D/ploidy gives the same numbers bit for bit
    X = np.asfortranarray(D.astype(np.float64) / ploidy)
    b2, y2, mu2, q2 = gbm.gblup_arrays(X, Y, lambda_=lam)
    assert q2 == q[0] and np.array_equal(y2, y_pred) and np.array_equal(b2, b_hat)
    # GRM entries and column statistics
    G, qg = gbm.grm(X)
    assert G.shape == (n, n) and qg == int(z["q"])
    assert rel(np.diag(G), z["G_diag"]) < 1e-12
    assert rel(G[0], z["G_first_row"]) < 1e-12
    assert abs(np.trace(G) - float(z["G_trace"])) < 1e-12 * abs(float(z["G_trace"]))
    assert abs(G.sum() - float(z["G_sum"])) < 1e-9 * np.abs(G).sum()
    m, s, k, _ = gbm.colstats(X)
    assert np.array_equal(k, z["keep"]) and rel(m, z["mean"]) < 1e-14 and rel(s[k], z["sd"][k]) < 1e-13


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_golden_fixture_model_function(path):
    """gblup(; genomes, phenomes) on the full fixture (missing phenotypes included): the
    extractxyetc filter drops them, and Fit matches the stored fit and metrics."""
    z = np.load(path)
    D, ploidy, Yfull = z["dosage"], int(z["ploidy"]), z["phenotypes"]
    n, p = D.shape
    X = D.astype(np.float64) / ploidy
    ent = [f"entry_{i}" for i in range(n)]
    loci = [f"chr1\t{j}\tA|T\tA" for j in range(p)]
    g = gbm.Genomes(ent, ["pop"] * n, loci, X)
    ph = gbm.Phenomes(ent, ["pop"] * n, [f"trait_{k + 1}" for k in range(Yfull.shape[1])], Yfull)
    met = json.loads(str(z["metrics_json"]))
    for k in range(Yfull.shape[1]):
        fit = gbm.gblup(genomes=g, phenomes=ph, idx_trait=k + 1, lambda_=float(z["lam"]))
        assert fit.checkdims() and fit.model == "gblup"
        assert fit.entries == [e for e, keep in zip(ent, z["keep_rows"]) if keep]
        assert rel(fit.y_pred, z["y_pred"][:, k]) < TOL_TIGHT
        assert rel(fit.b_hat, z["b_hat"][:, k]) < TOL_CONTRACT
        for key, v in met[k].items():
            assert abs(fit.metrics[key] - v) < 1e-8 * max(1.0, abs(v)), key


def test_gwasprep_doctest_moments_on_device():
    """src/gwas.jl:53-62: every kept standardised column has |mean| < 1e-10 and |std − 1| <
    1e-10 (ddof = 1) — on the Z the HIP standardise kernel writes."""
    from gbm.sharded import HipShardStages
    n, p = 333, 1777
    X = oracle.synth_genotypes(7, n, p)
    X[:, 0] = 0.0  # monomorphic: dropped (sd <= eps)
    st = HipShardStages(n, p, device=0)
    st.upload_genotypes(X)
    st.standardize()
    Z = st.Z[:, :n].cpu().numpy()
    keep = st.keep.cpu().numpy() != 0
    assert not keep[0] and int(st.q.item()) == keep.sum() == p - 1
    Zk = Z[keep]
    assert np.abs(Zk.mean(axis=1)).max() < 1e-10
    assert np.abs(Zk.std(axis=1, ddof=1) - 1.0).max() < 1e-10


def _related_population(seed, n=100, p=10000, founders=6, ploidy=4, block=1000):
    """simulategenomes-like data (tetraploid allele frequencies d/4, LD blocks copied from a few
    founder haplotypes, so entries are related)."""
    rng = np.random.default_rng(seed)
    f = rng.uniform(0.05, 0.5, p)
    F = (rng.random((founders * ploidy, p)) < f).astype(np.float64)
    X = np.zeros((n, p))
    cols = np.arange(p)
    for i in range(n):
        for _ in range(ploidy):
            src = rng.integers(0, founders * ploidy, size=-(-p // block))
            X[i] += F[src[cols // block], cols]
    return np.asfortranarray(X / ploidy)


def test_predict_doctest_shape():
    """src/prediction.jl:175-186: fit on entries 1:90, predict 91:100, cor > 0.5 (the doctest's
    check on its seeded simulated population; here a seeded related population of the same
    shape), with the HIP fit equal to the oracle's."""
    X = _related_population(0)
    Y = oracle.synth_phenotypes(X, 1, qtl_frac=0.1, h2=0.8)
    n, p = X.shape
    ent = [f"entry_{i}" for i in range(n)]
    g = gbm.Genomes(ent, ["pop"] * n, [f"l{j}" for j in range(p)], X)
    ph = gbm.Phenomes(ent, ["pop"] * n, ["trait_1"], Y)
    fit = gbm.gblup(genomes=g, phenomes=ph, idx_entries=list(range(1, 91)))
    y_hat = gbm.predict(fit, g, list(range(91, 101)))
    assert len(y_hat) == 10
    ref = oracle.gblup_fit(X[:90], Y[:90], 1.0)
    assert rel(fit.y_pred, ref["y_pred"][:, 0]) < TOL_TIGHT
    assert rel(y_hat, oracle.predict_linear(X[90:], ref["b_hat"])[:, 0]) < TOL_TIGHT
    assert np.corrcoef(Y[90:, 0], y_hat)[0, 1] > 0.5


# ---- GRM accumulation modes, forced per call ---------------------------------------------------

def _ws_bytes(n, p):
    return gbm.load_library().gbm_dev_grm_workspace(n, p)


@pytest.mark.parametrize("n,p", [(1030, 1234), (4999, 600), (1100, 2049), (700, 5000)])
@pytest.mark.parametrize("persist", ["1", "0"])
def test_grm_carry_mode_matches_oracle(gbm_env, n, p, persist):
    """In-order carry accumulation (unit (s, t) waits for (s−1, t)'s flag, adds its partial to
    the running tile in G): used automatically when the slabs would exceed 4 GiB (n ≳ 13 000);
    forced here with four loci ranges on ragged shapes. Also the slab mode with hardware
    dispatch (GBM_GRM_PERSIST=0)."""
    X = oracle.synth_genotypes(n * 7 + p, n, p)
    Gr, qr = oracle.grm(X)
    gbm_env.setenv("GBM_GRM_SPLIT", "4,2,1,1")
    gbm_env.setenv("GBM_GRM_PERSIST", persist)
    gbm_env.setenv("GBM_GRM_CARRY", "0")
    slab_ws = _ws_bytes(n, p)
    G0, q0 = gbm.grm(X)
    gbm_env.setenv("GBM_GRM_CARRY", "1")
    carry_ws = _ws_bytes(n, p)
    assert carry_ws < slab_ws  # carry mode: tile flags instead of the loci-range slabs
    assert gbm.load_library().gbm_dev_grm_slices(n, p) == 4
    G1, q1 = gbm.grm(X)
    assert q0 == q1 == qr
    assert rel(G0, Gr) < 1e-12 and rel(G1, Gr) < 1e-12
    assert np.array_equal(G1, G1.T)
    # same summation order (((P0 + P1) + P2) + P3) in both modes
    assert np.array_equal(G0, G1)


def test_gblup_carry_mode_matches_oracle(gbm_env):
    gbm_env.setenv("GBM_GRM_CARRY", "1")
    gbm_env.setenv("GBM_GRM_SPLIT", "5,3,1")
    n, p = 1030, 3000
    X = oracle.synth_genotypes(5, n, p)
    Y = oracle.synth_phenotypes(X, 6, ntraits=2)
    b_hat, y_pred, mu, q = gbm.gblup_arrays(X, Y, lambda_=1.0)
    ref = oracle.gblup_fit(X, Y, 1.0)
    assert q == ref["q"] and rel(y_pred, ref["y_pred"]) < TOL_TIGHT and rel(b_hat, ref["b_hat"]) < TOL_CONTRACT


def test_grm_carry_timeout_is_reported(gbm_env):
    """A timed-out inter-workgroup wait sets the carry error cell (int32 after the ntiles tile
    flags) to −1; gbm_dev_grm_reduce reads it back and fails instead of returning a wrong G.
    The cell is poisoned between the two stages to exercise that check."""
    import torch
    gbm_env.setenv("GBM_GRM_CARRY", "1")
    gbm_env.setenv("GBM_GRM_SPLIT", "1,1")
    gbm_env.setenv("GBM_GRM_EDGE", "0")
    lib = gbm.load_library()
    n, p = 640, 512
    npad, gdim = lib.gbm_dev_npad(n), lib.gbm_dev_gdim(n)
    X = oracle.synth_genotypes(3, n, p)
    Zt = torch.zeros((p, npad), dtype=torch.float64, device="cuda:0")
    m, s, k = oracle.colstats(X)
    assert k.all()
    Zt[:, :n] = torch.from_numpy(np.ascontiguousarray(oracle.standardize(X, m, s, k).T))
    G = torch.zeros((gdim, gdim), dtype=torch.float64, device="cuda:0")
    wsb = lib.gbm_dev_grm_workspace(n, p)
    ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda:0")
    stream = ctypes.c_void_p(torch.cuda.current_stream(0).cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    _lib.check(lib.gbm_dev_grm_syrk(P(Zt), npad, p, n, P(G), gdim, P(ws), wsb, stream), "syrk")
    _lib.check(lib.gbm_dev_grm_reduce(n, p, P(G), gdim, P(ws), stream), "reduce")  # clean run passes
    nt = npad // 128
    ws.view(torch.int32)[nt * (nt + 1) // 2] = -1
    rc = lib.gbm_dev_grm_reduce(n, p, P(G), gdim, P(ws), stream)
    assert rc == _lib.GBM_E_HIP and "timed out" in _lib.last_error()
