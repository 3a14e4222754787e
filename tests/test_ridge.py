"""Ridge path of reference ``ridge`` (GLMNet alpha = 0; src/linear.jl:162-239) — SURVEY.md §8f
row 4. CPU: the oracle's exact ridge against R-glmnet known answers (tests/golden/
glmnet_ridge_r.npz) and the selection quirks. GPU: the session ridge path vs the oracle and vs the
same known answers. glmnet divides the user λ by the population sd of y (elnet's vlam = ulam/ys),
so the exact minimiser matches R to ~5e-8 (the fixture's coefficients are printed to 7-8 digits);
the y-scaled cases pin that σ_y factor: glmnet(X, c·y, c·λ) = c·glmnet(X, y, λ)."""
import os

import numpy as np
import pytest

import gbm
import oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "glmnet_ridge_r.npz")


def _cases():
    z = np.load(GOLD)
    data = z["data"]
    for c in z["cases"]:
        n, p, lam = int(c[0]), int(c[1]), float(c[3])
        y = data[:n, 0] - data[:n, 0].mean()
        y /= y.std(ddof=1)
        X = data[:n, 1:p + 1] - data[:n, 1:p + 1].mean(axis=0)
        X /= X.std(axis=0, ddof=1)
        yield X, y, lam, c[4:4 + p]


def test_oracle_ridge_matches_r_glmnet():
    m = 0
    for X, y, lam, ref in _cases():
        a0, b = oracle.ridge_exact(X, y, lam)
        assert np.abs(b - ref).max() < 1e-6, (lam, b, ref)
        assert abs(a0) < 1e-12
        for c in (10.0, 0.1):  # σ_y ≠ 1: the same R answers, scaled
            a0c, bc = oracle.ridge_exact(X, c * y, c * lam)
            assert np.abs(bc / c - ref).max() < 1e-6, (c, lam)
        m += 1
    assert m == 27


def test_ridge_select_quirks():
    a0 = np.array([10.0, 20.0, 30.0, 40.0])
    betas = np.array([[0.0, 1.0, 2.0, 0.0], [0.0, 3.0, 5.0, 0.0]])
    loss = np.array([0.1, 0.3, 0.2, 0.4])  # sorted: 0, 2, 1, 3
    b = gbm.ridge_select(a0, betas, loss)
    # λ #1 has zero slopes (variance < 1e-10): skipped; the next by loss is λ #3 (idx 2), and its
    # intercept is a0[idx_sort][idx_sort[1]] = a0[idx_sort][2] = a0[1] (src/linear.jl:215,220)
    assert np.array_equal(b, [20.0, 2.0, 5.0])


def test_glmnet_folds_balanced():
    f = gbm.glmnet_folds(23, 7, np.random.default_rng(0))
    assert sorted(np.bincount(f)[1:]) == [3, 3, 3, 3, 3, 4, 4]


@pytest.mark.gpu
def test_gpu_ridge_path_matches_r_glmnet_and_oracle():
    for X, y, lam, ref in _cases():
        for c in (1.0, 10.0):
            with gbm.GenotypeSession(X) as s:
                b = s.ridge_path(np.arange(X.shape[0]), c * y, [c * lam])[:, 0]
            a0, bo = oracle.ridge_exact(X, c * y, c * lam)
            assert np.abs(b[1:] / c - ref).max() < 1e-6
            assert np.abs(b[1:] - bo).max() < 1e-9 * max(1.0, np.abs(bo).max())
            assert abs(b[0] - a0) < 1e-9 * c


@pytest.mark.gpu
def test_gpu_ridge_path_cv_matches_oracle():
    X = oracle.synth_genotypes(41, 200, 1000)  # config C1 shape
    y = oracle.synth_phenotypes(X, 42)[:, 0]
    got = gbm.ridge_path_cv(X, y, seed=3)
    folds = gbm.glmnet_folds(200, 10, np.random.default_rng(3))
    ref = oracle.ridge_path_cv(X, y, folds)
    rel = lambda a, b: np.abs(a - b).max() / np.abs(b).max()
    assert rel(got["lambda"], ref["lambda"]) < 1e-12
    assert rel(got["betas"], ref["betas"]) < 1e-8
    assert rel(got["a0"], ref["a0"]) < 1e-8
    assert rel(got["meanloss"], ref["meanloss"]) < 1e-8


@pytest.mark.gpu
def test_gpu_ridge_model_function():
    X = oracle.synth_genotypes(43, 150, 600)
    Y = oracle.synth_phenotypes(X, 44)
    ent = [f"e{i}" for i in range(150)]
    g = gbm.Genomes(ent, ["p"] * 150, [f"l{j}" for j in range(600)], X)
    ph = gbm.Phenomes(ent, ["p"] * 150, ["t"], Y)
    fit = gbm.ridge(genomes=g, phenomes=ph, seed=5)
    assert fit.model == "ridge" and fit.checkdims()
    folds = gbm.glmnet_folds(150, 10, np.random.default_rng(5))
    ref = oracle.ridge_path_cv(X, Y[:, 0], folds)
    b_ref = gbm.ridge_select(ref["a0"], ref["betas"], ref["meanloss"])
    assert np.abs(fit.b_hat - b_ref).max() < 1e-8 * np.abs(b_ref).max()
    assert fit.metrics["cor"] > 0.5  # the reference doctest (src/linear.jl:153-156)
