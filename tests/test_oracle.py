"""CPU tests of the oracle (test infrastructure): golden fixtures, the two restatements against
each other, the reference doctest properties and the known-answer identities."""
import ctypes
import glob
import json
import os

import numpy as np
import pytest

import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
# the GBLUP golden fixtures (make_golden.py); the R known-answer files have their own tests
GOLDEN = sorted(f for f in glob.glob(os.path.join(HERE, "golden", "*.npz"))
                if not f.endswith(("glmnet_ridge_r.npz", "lmer_r.npz")))


def rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(np.abs(np.asarray(b)).max(), 1e-300))


def load_case(path):
    z = np.load(path)  # allow_pickle=False (default)
    X = z["dosage"].astype(np.float64) / float(z["ploidy"])
    keep_rows = z["keep_rows"]
    Y = z["phenotypes"][keep_rows]
    return z, X[keep_rows], Y


def test_fixtures_present():
    assert len(GOLDEN) >= 3


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_numpy_oracle_reproduces_golden(path):
    z, X, Y = load_case(path)
    r = oracle.gblup_fit(X, Y, float(z["lam"]))
    assert r["q"] == int(z["q"])
    assert rel(r["y_pred"], z["y_pred"]) < 1e-12
    assert rel(r["b_hat"], z["b_hat"]) < 1e-10
    assert rel(r["mu"], z["mu"]) < 1e-12
    assert abs(np.trace(r["G"]) - float(z["G_trace"])) < 1e-9 * abs(float(z["G_trace"]))
    assert np.array_equal(r["keep"], z["keep"])
    met = json.loads(str(z["metrics_json"]))
    for t, m in enumerate(met):
        mm = oracle.metrics(Y[:, t], r["y_pred"][:, t])
        for k in m:
            assert abs(mm[k] - m[k]) <= 1e-10 * max(1.0, abs(m[k])), k


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_c_oracle_matches_golden(path, oracle_c):
    z, X, Y = load_case(path)
    n, p = X.shape
    t = Y.shape[1]
    Xf = np.asfortranarray(X)
    Yf = np.asfortranarray(Y)
    b_hat = np.zeros((p + 1, t), order="F")
    y_pred = np.zeros((n, t), order="F")
    mu = np.zeros(t)
    q = np.zeros(1, dtype=np.int64)
    rc = oracle_c.gbm_ref_gblup_fit(Xf.ctypes.data, n, p, n, Yf.ctypes.data, n, t, float(z["lam"]),
                                    b_hat.ctypes.data, y_pred.ctypes.data, mu.ctypes.data, q.ctypes.data)
    assert rc == 0
    assert q[0] == int(z["q"])
    assert rel(y_pred, z["y_pred"]) < 1e-11
    assert rel(b_hat, z["b_hat"]) < 1e-9
    G = np.zeros((n, n), order="F")
    assert oracle_c.gbm_ref_grm(Xf.ctypes.data, n, p, n, G.ctypes.data, n) == int(z["q"])
    assert abs(np.trace(G) - float(z["G_trace"])) < 1e-9 * abs(float(z["G_trace"]))
    assert rel(G[0], z["G_first_row"]) < 1e-12


def test_generator_c_equals_numpy(oracle_c):
    n, p, j0 = 97, 131, 12345
    X = oracle.synth_genotypes(4242, n, p, j0=j0)
    Xc = np.zeros((n, p), order="F")
    oracle_c.gbm_ref_synth_matrix(4242, n, p, j0, Xc.ctypes.data, n)
    assert np.array_equal(X, Xc)
    # MAF thresholds in [0.05, 0.5): allele frequencies of dosage/2 near f
    Xb = oracle.synth_genotypes(1, 4000, 50)
    f = Xb.mean(axis=0)
    assert np.all(f > 0.02) and np.all(f < 0.55)
    assert set(np.unique(Xb)) <= {0.0, 0.5, 1.0}


def test_doctest_standardisation_moments():
    """reference src/gwas.jl:55-62: standardised columns have mean 0 and std 1 within 1e-10."""
    X = oracle.synth_genotypes(3, 120, 300)
    m, s, keep = oracle.colstats(X)
    Z = oracle.standardize(X, m, s, keep)
    assert np.all(np.abs(Z.mean(axis=0)) < 1e-10)
    assert np.all(np.abs(Z.std(axis=0, ddof=1) - 1.0) < 1e-10)


def test_primal_dual_identity():
    """RR-BLUP primal (ZᵀZ + qλI)β = Zᵀ(y − μ̂) equals the dual GBLUP marker effects."""
    X = oracle.synth_genotypes(8, 150, 400)
    y = oracle.synth_phenotypes(X, 1)[:, 0]
    for lam in (0.3, 1.0, 4.0):
        r = oracle.gblup_fit(X, y, lam)
        beta = oracle.rrblup_primal(X, y, lam, r["mu"][0])
        keep, s = r["keep"], r["sd"]
        assert rel(beta, r["b_hat"][1:, 0][keep] * s[keep]) < 1e-10
        assert rel(oracle.predict_linear(X, r["b_hat"][:, 0]), r["y_pred"][:, 0]) < 1e-12


def test_gls_intercept_matches_explicit_inverse():
    """μ̂ = 1ᵀV⁻¹y/1ᵀV⁻¹1 with V⁻¹ from an explicit pinv (the reference's route, src/gwas.jl:595-596)."""
    X = oracle.synth_genotypes(4, 80, 200)
    y = oracle.synth_phenotypes(X, 2)[:, 0]
    r = oracle.gblup_fit(X, y, 1.0)
    Vi = np.linalg.pinv(r["G"] + np.eye(80))
    one = np.ones(80)
    mu = (one @ Vi @ y) / (one @ Vi @ one)
    assert abs(mu - r["mu"][0]) < 1e-10 * max(1, abs(mu))
    a = Vi @ (y - mu)
    assert rel(r["a"][:, 0], a) < 1e-9


def test_gebv_correlation_doctest_property():
    """Qualitative reference doctest (src/linear.jl:153-159): in-sample cor > 0.5 at h² = 0.5."""
    X = oracle.synth_genotypes(10, 200, 1000)
    y = oracle.synth_phenotypes(X, 5)[:, 0]
    r = oracle.gblup_fit(X, y, 1.0)
    assert oracle.metrics(y, r["y_pred"][:, 0])["cor"] > 0.5


def test_ploidy_aware_grm_restatement():
    """The ploidy-aware GRM restatement (Core's grmploidyaware is un-vendored: parity unpinned)
    against VanRaden's method 1 written directly on 0/1/2 dosages (Z = M − 2p, G = ZZᵀ / (2Σp(1−p)))
    and, for ploidy 4, an element-wise loop; the reference's ploidy inference (src/gwas.jl:119) on
    the doctest's rounding of frequencies to k/4 (src/gwas.jl:43-45)."""
    import gbm
    rng = np.random.default_rng(5)
    M = rng.integers(0, 3, size=(40, 90)).astype(np.float64)
    M[:, 7] = 1.0  # monomorphic: contributes nothing
    G, den = oracle.grm_ploidy_aware(M / 2.0, 2)
    p = M.mean(axis=0) / 2.0
    Z = M - 2.0 * p
    assert np.allclose(G, Z @ Z.T / (2.0 * (p * (1.0 - p)).sum()), rtol=1e-13, atol=1e-13)
    X4 = np.round(rng.random((12, 30)) * 4.0) / 4.0
    G4, den4 = oracle.grm_ploidy_aware(X4, 4)
    f = X4.mean(axis=0)
    want = np.array([[sum(4 * (X4[i, j] - f[j]) * 4 * (X4[k, j] - f[j]) for j in range(30)) for k in range(12)]
                     for i in range(12)]) / (4.0 * (f * (1 - f)).sum())
    assert np.allclose(G4, want, rtol=1e-12, atol=1e-12)
    assert gbm.infer_ploidy(X4) == 4 and gbm.infer_ploidy(M / 2.0) == 2
