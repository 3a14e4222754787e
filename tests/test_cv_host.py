"""CPU tests of the cross-validation host layer (job setup of reference cvbulk,
src/cross_validation.jl:268-401) and of the REML algebra libgbm uses (the profile form of the
reference's loglikreml, src/gwas.jl:450-483) — no GPU needed."""
import functools

import numpy as np
import pytest

import gbm
import oracle
from gbm.cv import _gblup_lambda


def _data(n=60, p=80, t=2, seed=3, missing=True):
    X = oracle.synth_genotypes(seed, n, p)
    Y = oracle.synth_phenotypes(X, seed + 1, ntraits=t)
    if missing:
        Y[[1, 7, 13], 0] = np.nan
    ent = [f"entry_{i}" for i in range(n)]
    pops = [f"pop_{i % 3}" for i in range(n)]
    g = gbm.Genomes(ent, pops, [f"l{j}" for j in range(p)], X)
    ph = gbm.Phenomes(ent, pops, [f"trait_{k + 1}" for k in range(t)], Y)
    return g, ph


def test_fold_assignments_reproducible_and_in_range():
    a = gbm.fold_assignments(50, 5, 3, 2, 42)
    b = gbm.fold_assignments(50, 5, 3, 2, 42)
    assert a.shape == (2, 3, 50) and np.array_equal(a, b)
    assert a.min() >= 1 and a.max() <= 5
    assert not np.array_equal(a[0, 0], a[1, 0])  # independent draws per trait (src/cross_validation.jl:359)


def test_cvbulk_setup_jobs_notes_and_no_leakage():
    g, ph = _data()
    models = [gbm.gblup, functools.partial(gbm.gblup, lambda_=2.0)]
    cvs, notes, mv = gbm.cvbulk_setup(genomes=g, phenomes=ph, models=models, n_replications=2, n_folds=3, seed=1)
    assert len(cvs) == len(mv) == 2 * 2 * 3 * 2 - len(notes) * 2
    for cv in cvs:
        assert not set(cv.fit.entries) & set(cv.validation_entries)
        assert cv.fit.b_hat_labels[0] == "intercept" and len(cv.fit.b_hat_labels) == 81
        assert cv.checkdims()
    # trait_1's missing entries never appear
    miss = {"entry_1", "entry_7", "entry_13"}
    for cv in cvs:
        if cv.fit.trait == "trait_1":
            assert not (set(cv.fit.entries) | set(cv.validation_entries)) & miss


def test_cvbulk_setup_notes_for_degenerate_folds():
    g, ph = _data(n=20, missing=False)
    ph.phenotypes[:, 1] = 3.0  # zero variance
    cvs, notes, _ = gbm.cvbulk_setup(genomes=g, phenomes=ph, n_replications=1, n_folds=2, seed=0)
    assert any(s.startswith("zero_variance;trait_2") for s in notes)
    ph.phenotypes[:, 0] = np.nan
    ph.phenotypes[:2, 0] = 1.0
    _, notes, _ = gbm.cvbulk_setup(genomes=g, phenomes=ph, n_replications=1, n_folds=2, seed=0)
    assert any(s.startswith("too_many_missing;trait_1") for s in notes)


def test_cvbulk_setup_argument_errors():
    g, ph = _data()
    with pytest.raises(gbm.ArgumentError):
        gbm.cvbulk_setup(genomes=g, phenomes=ph, n_folds=0)
    with pytest.raises(gbm.ArgumentError):
        gbm.cvbulk_setup(genomes=g, phenomes=ph, n_replications=101)
    with pytest.raises(gbm.ArgumentError):
        gbm.cvbulk_setup(genomes=g, phenomes=ph, models=[])
    ph2 = gbm.Phenomes(list(reversed(ph.entries)), ph.populations, ph.traits, ph.phenotypes)
    with pytest.raises(gbm.ArgumentError):
        gbm.cvbulk_setup(genomes=g, phenomes=ph2)


def test_gblup_model_recognition():
    assert _gblup_lambda(gbm.gblup) == 1.0
    assert _gblup_lambda(functools.partial(gbm.gblup, lambda_=3.0)) == 3.0
    assert _gblup_lambda(functools.partial(gbm.gblup, lambda_="reml")) == "reml"
    assert _gblup_lambda(functools.partial(gbm.gblup, verbose=True)) is None
    assert _gblup_lambda(len) is None


def test_reml_profile_algebra_matches_loglikreml():
    """libgbm evaluates loglikreml from one Cholesky of G + λI: logdet, 1ᵀV⁻¹1, 1ᵀV⁻¹y, yᵀV⁻¹y
    (session.cpp reml_objective). Check that algebra against the pinv restatement."""
    X = oracle.synth_genotypes(9, 80, 300)
    y = oracle.synth_phenotypes(X, 10)[:, 0]
    G, _ = oracle.grm(X)
    one = np.ones(80)
    for s2e, s2u in [(0.5, 0.5), (0.2, 0.9), (1e-3, 0.7), (0.9, 1e-2)]:
        lam = s2e / s2u
        L = np.linalg.cholesky(G + lam * np.eye(80))
        w1, wy = np.linalg.solve(L, one), np.linalg.solve(L, y)
        logdet = 2 * np.log(np.diag(L)).sum()
        c11, c1y, yy = w1 @ w1, w1 @ wy, wy @ wy
        Q = yy - c1y ** 2 / c11
        f = 0.5 * (80 * np.log(s2u) + logdet) + Q / s2u + np.log(c11) - np.log(s2u)
        ref = oracle.loglikreml([s2e, s2u], y, one[:, None], G)
        assert abs(f - ref) < 1e-9 * max(1.0, abs(ref))
