"""Device genotype sessions (fold farming + GRM cache, REML λ) and GPU cross-validation vs the
oracle — SURVEY.md §8f rows 1-2. Fold fits are pinned to the oracle's GBLUP on the same training
rows; the REML objective to the line-for-line restatement of reference loglikreml
(src/gwas.jl:450-483); the REML optimum to an L-BFGS-B run of that objective over the reference's
box (src/gwas.jl:577-590)."""
import functools

import numpy as np
import pytest

import gbm
import oracle

pytestmark = pytest.mark.gpu


def rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(np.abs(np.asarray(b)).max(), 1e-300))


@pytest.fixture(scope="module")
def data():
    X = oracle.synth_genotypes(21, 300, 1500)
    Y = oracle.synth_phenotypes(X, 22, ntraits=3)
    return X, Y


def test_session_fit_on_subset_matches_oracle_and_caches(data):
    X, Y = data
    idx = np.sort(np.random.default_rng(0).choice(300, 230, replace=False))
    with gbm.GenotypeSession(X) as s:
        b1, yp1, mu1, q1 = s.gblup(idx, Y[idx, :2], 1.0)
        ref = oracle.gblup_fit(X[idx], Y[idx, :2], 1.0)
        assert q1 == ref["q"]
        assert rel(yp1, ref["y_pred"]) < 1e-9 and rel(mu1, ref["mu"]) < 1e-9 and rel(b1, ref["b_hat"]) < 1e-6
        assert s.stats() == (1, 0)
        # same training set, another λ and trait: cache hit, no second GRM
        b2, yp2, _, _ = s.gblup(idx, Y[idx, 2], 0.5)
        assert s.stats() == (1, 1)
        assert rel(yp2, oracle.gblup_fit(X[idx], Y[idx, 2], 0.5)["y_pred"]) < 1e-9
        # repeat is bit-identical
        b3, yp3, _, _ = s.gblup(idx, Y[idx, :2], 1.0)
        assert np.array_equal(yp1, yp3) and np.array_equal(b1, b3)
        # predict on held-out rows (reference predict, src/prediction.jl:228)
        val = np.setdiff1d(np.arange(300), idx)
        assert rel(s.predict(val, b1[:, 0]), oracle.predict_linear(X[val], b1[:, 0])) < 1e-12
        # another training set rebuilds
        s.gblup(idx[:-5], Y[idx[:-5], 0], 1.0)
        assert s.stats() == (2, 2)


def test_session_argument_errors(data):
    X, Y = data
    with gbm.GenotypeSession(X) as s:
        with pytest.raises(gbm.ArgumentError, match="increasing"):
            s.gblup(np.array([3, 2, 5]), Y[[3, 2, 5], 0])
        with pytest.raises(gbm.ArgumentError, match="out of range"):
            s.gblup(np.array([0, 1, 400]), Y[:3, 0])
        with pytest.raises(gbm.GBMError, match="variance"):
            s.gblup(np.arange(10), np.ones(10))


def test_session_dosage_i8_matches_f64(data):
    X, Y = data
    D = np.rint(X * 2).astype(np.int8)
    idx = np.arange(0, 300, 2)
    with gbm.GenotypeSession(X) as a, gbm.GenotypeSession(dosage_i8=D, ploidy=2) as b:
        ra, rb = a.gblup(idx, Y[idx, 0]), b.gblup(idx, Y[idx, 0])
        assert np.array_equal(ra[1], rb[1])


def test_reml_objective_matches_loglikreml(data):
    X, Y = data
    idx = np.arange(0, 300, 3)
    G, _ = oracle.grm(X[idx])
    y = Y[idx, 0]
    th = np.array([(0.5, 0.5), (0.2, 0.9), (1e-3, 0.7), (0.9, 1e-2), (1.0, 1.0)])
    with gbm.GenotypeSession(X) as s:
        got = s.reml_objective(idx, y, th[:, 0], th[:, 1])
    ref = [oracle.loglikreml(t, y, np.ones((idx.size, 1)), G) for t in th]
    assert rel(got, ref) < 1e-9


def test_reml_optimum_at_least_as_good_as_reference_optimiser(data):
    X, Y = data
    idx = np.arange(250)
    G, _ = oracle.grm(X[idx])
    ref = oracle.reml_reference(Y[idx, 1], G)
    with gbm.GenotypeSession(X) as s:
        r = s.reml(idx, Y[idx, 1])
        f_at_ref = s.reml_objective(idx, ref["y_std"], [ref["sigma2_e"]], [ref["sigma2_u"]])[0]
    assert abs(f_at_ref - ref["objective"]) < 1e-8 * max(1.0, abs(ref["objective"]))
    assert r["objective"] <= ref["objective"] + 1e-7 * max(1.0, abs(ref["objective"]))
    assert abs(np.log(r["lambda"]) - np.log(ref["lambda"])) < 1e-2
    assert 0 < r["sigma2_u"] <= 1 and 0 < r["sigma2_e"] <= 1


def test_gblup_reml_option(data):
    X, Y = data
    n = 200
    g = gbm.Genomes([f"e{i}" for i in range(n)], ["p"] * n, [f"l{j}" for j in range(X.shape[1])], X[:n])
    ph = gbm.Phenomes(g.entries, g.populations, ["t1"], Y[:n, :1])
    fit = gbm.gblup(genomes=g, phenomes=ph, lambda_="reml")
    lam = fit.metrics_reml["lambda"]
    assert rel(fit.y_pred, oracle.gblup_fit(X[:n], Y[:n, 0], lam)["y_pred"][:, 0]) < 1e-9


def _cv_inputs():
    X = oracle.synth_genotypes(31, 150, 700)
    Y = oracle.synth_phenotypes(X, 32, ntraits=2)
    Y[[4, 40, 99], 1] = np.nan
    ent = [f"entry_{i}" for i in range(150)]
    pops = [f"pop_{i % 2}" for i in range(150)]
    return (gbm.Genomes(ent, pops, [f"l{j}" for j in range(700)], X),
            gbm.Phenomes(ent, pops, ["trait_1", "trait_2"], Y))


@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_cvbulk_gpu_matches_oracle_per_fold(devices):
    g, ph = _cv_inputs()
    X, Y = g.allele_frequencies, ph.phenotypes
    models = [gbm.gblup, functools.partial(gbm.gblup, lambda_=2.5)]
    cvs, notes = gbm.cvbulk(genomes=g, phenomes=ph, models=models, n_replications=2, n_folds=3, seed=5,
                            devices=devices)
    assert len(cvs) == 2 * 2 * 3 * 2 and not notes
    pos = {e: i for i, e in enumerate(g.entries)}
    for i, cv in enumerate(cvs):
        tr = np.array(sorted(pos[e] for e in cv.fit.entries))
        va = np.array([pos[e] for e in cv.validation_entries])
        t = ph.traits.index(cv.fit.trait)
        # models alternate gblup (λ=1), partial (λ=2.5) within each fold
        k = i % 2
        ref = oracle.gblup_fit(X[tr], Y[tr, t], [1.0, 2.5][k])
        assert rel(cv.fit.y_pred, ref["y_pred"][:, 0]) < 1e-9
        assert rel(cv.validation_y_pred, oracle.predict_linear(X[va], ref["b_hat"][:, 0])) < 1e-8
        assert np.allclose(cv.validation_y_true, Y[va, t])
        assert set(cv.metrics) == set(oracle.metrics(Y[va, t], cv.validation_y_pred))


def test_cvmultithread_shuffled_entries_and_missing_training_phenotypes():
    """cvmultithread! takes CVs whose entries come in any order and whose training phenotypes may
    be missing (extractxyetc drops those rows, src/prediction.jl:114-131): Fit.entries, y_true and
    y_pred keep the caller's order, validation predictions keep the validation order."""
    g, ph = _cv_inputs()
    X = g.allele_frequencies
    cvs, notes, mv = gbm.cvbulk_setup(genomes=g, phenomes=ph, models=[gbm.gblup], n_replications=1,
                                      n_folds=3, seed=7)
    rng = np.random.default_rng(0)
    for cv in cvs:
        k = rng.permutation(len(cv.fit.entries))
        cv.fit.entries = [cv.fit.entries[j] for j in k]
        cv.fit.populations = [cv.fit.populations[j] for j in k]
        k = rng.permutation(len(cv.validation_entries))
        cv.validation_entries = [cv.validation_entries[j] for j in k]
    Y = ph.phenotypes.copy()
    pos = {e: i for i, e in enumerate(g.entries)}
    drop = [pos[cvs[0].fit.entries[3]], pos[cvs[0].fit.entries[10]]]
    ph.phenotypes[drop, ph.traits.index(cvs[0].fit.trait)] = np.inf  # missing after setup
    entries_before = [list(cv.fit.entries) for cv in cvs]
    gbm.cvmultithread(cvs, genomes=g, phenomes=ph, models_vector=mv, devices=[0])
    for cv, before in zip(cvs, entries_before):
        t = ph.traits.index(cv.fit.trait)
        rows = [pos[e] for e in before if np.isfinite(ph.phenotypes[pos[e], t])]
        assert [pos[e] for e in cv.fit.entries] == rows
        assert np.array_equal(cv.fit.y_true, ph.phenotypes[rows, t])
        ref = oracle.gblup_fit(X[rows], ph.phenotypes[rows, t], 1.0)
        assert rel(cv.fit.y_pred, ref["y_pred"][:, 0]) < 1e-9
        va = [pos[e] for e in cv.validation_entries]
        assert rel(cv.validation_y_pred, oracle.predict_linear(X[va], ref["b_hat"][:, 0])) < 1e-8
    assert len(cvs[0].fit.entries) == len(entries_before[0]) - 2
    ph.phenotypes[:] = Y


def test_validate_mirrors_reference():
    g, ph = _cv_inputs()
    fit = gbm.gblup(genomes=g, phenomes=ph, idx_entries=list(range(1, 101)))
    cv = gbm.validate(fit, g, ph, idx_validation=list(range(101, 151)), replication="r", fold="f")
    assert cv.checkdims() and cv.fold == "f"
    with pytest.raises(gbm.ArgumentError, match="leakage"):
        gbm.validate(fit, g, ph, idx_validation=[5, 120])


def test_synthetic_session_matches_host_session(data):
    """gbm_session_create_synthetic: X generated on the device is the oracle's synthetic X, so the
    session fits equal the oracle's on the same rows; gbm.synth's host copy is bit-exact."""
    from gbm import synth
    X = oracle.synth_genotypes(4242, 257, 700)
    assert np.array_equal(synth.genotypes(4242, 257, 700), X)
    assert np.array_equal(synth.genotypes(4242, 257, 300, j0=400), X[:, 400:])
    Y = oracle.synth_phenotypes(X, 5, ntraits=2)
    idx = np.arange(0, 257, 2)
    with gbm.GenotypeSession.synthetic(4242, 257, 700) as s:
        b, yp, mu, q = s.gblup(idx, Y[idx], 1.0)
    ref = oracle.gblup_fit(X[idx], Y[idx], 1.0)
    assert q == ref["q"]
    assert rel(yp, ref["y_pred"]) < 1e-9 and rel(b, ref["b_hat"]) < 1e-6


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_cabi_reml_fit_matches_session_reml_and_oracle(data, devices):
    """gbm_gblup_fit_reml (the drop-in gblup(λ = :reml); VERDICT r02 Missing #3): per trait the REML
    λ on the call's own GRM equals gbm_session_reml's on the same rows (same objective, same search:
    the GRMs agree to rounding, the λ to 1e-9), reaches the oracle's loglikreml optimum
    (src/gwas.jl:450-483,577-590), and each trait's fit is the oracle's GBLUP at its λ."""
    X, Y = data
    idx = np.arange(260)
    Xs, Ys = X[idx], Y[idx]
    b, yp, mu, q, r = gbm.gblup_reml_arrays(Xs, Ys, devices=devices)
    G, _ = oracle.grm(Xs)
    with gbm.GenotypeSession(X) as s:
        for t in range(Ys.shape[1]):
            rs = s.reml(idx, Ys[:, t])
            assert abs(np.log(r["lambda"][t]) - np.log(rs["lambda"])) < 1e-9
            assert abs(r["sigma2_u"][t] - rs["sigma2_u"]) < 1e-9 * rs["sigma2_u"]
            assert abs(r["sigma2_e"][t] - rs["sigma2_e"]) < 1e-9 * rs["sigma2_e"]
            ref = oracle.reml_reference(Ys[:, t], G)
            assert abs(np.log(r["lambda"][t]) - np.log(ref["lambda"])) < 1e-2
            f_got = oracle.loglikreml((r["sigma2_e"][t], r["sigma2_u"][t]), ref["y_std"], np.ones((idx.size, 1)), G)
            assert f_got <= ref["objective"] + 1e-7 * max(1.0, abs(ref["objective"]))
            fit = oracle.gblup_fit(Xs, Ys[:, t], r["lambda"][t])
            assert q == fit["q"]
            assert rel(yp[:, t], fit["y_pred"][:, 0]) < 1e-9 and abs(mu[t] - fit["mu"][0]) < 1e-9 * abs(fit["mu"][0])
            assert rel(b[:, t], fit["b_hat"][:, 0]) < 1e-6
    # the model function takes the same route
    g = gbm.Genomes([f"e{i}" for i in idx], ["p"] * idx.size, [f"l{j}" for j in range(X.shape[1])], Xs)
    ph = gbm.Phenomes(g.entries, g.populations, ["t1"], Ys[:, :1])
    f1 = gbm.gblup(genomes=g, phenomes=ph, lambda_="reml", devices=devices, grm=None)  # the same GRM mode as r
    assert f1.metrics_reml["lambda"] == r["lambda"][0] and np.array_equal(f1.y_pred, yp[:, 0])
