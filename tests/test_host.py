"""CPU tests of the host mirror of the reference interface: extractxyetc (src/prediction.jl:53-139),
predict's checks (src/prediction.jl:189-235), Fit, metrics (src/metrics.jl)."""
import numpy as np
import pytest

import gbm
import oracle


def make_data(n=40, p=60, t=2, seed=0):
    rng = np.random.default_rng(seed)
    X = oracle.synth_genotypes(seed, n, p)
    Y = rng.standard_normal((n, t))
    entries = [f"entry_{i}" for i in range(n)]
    pops = [f"pop_{i % 3}" for i in range(n)]
    loci = [f"chr1\t{j}\tA|T\tA" for j in range(p)]
    return gbm.Genomes(entries, pops, loci, X), gbm.Phenomes(entries, pops, [f"trait_{k}" for k in range(t)], Y)


def test_extractxyetc_doctest_properties():
    """src/prediction.jl:44-50: X == hcat(ones, allele_frequencies), y == phenotypes[:, 1]."""
    g, ph = make_data()
    X, y, entries, pops, loci = gbm.extractxyetc(g, ph)
    assert np.array_equal(X, np.hstack([np.ones((40, 1)), g.allele_frequencies]))
    assert np.array_equal(y, ph.phenotypes[:, 0])
    assert entries == g.entries and loci == g.loci_alleles and pops == g.populations
    X2, *_ = gbm.extractxyetc(g, ph, add_intercept=False)
    assert np.array_equal(X2, g.allele_frequencies) and X2.flags.f_contiguous


def test_extractxyetc_subsets_and_missing():
    g, ph = make_data()
    ph.phenotypes[3, 1] = np.nan
    ph.phenotypes[5, 1] = np.inf
    idx_e = np.array([1, 2, 4, 5, 6, 9])  # 1-based
    idx_l = np.array([2, 3, 10])
    X, y, entries, pops, loci = gbm.extractxyetc(g, ph, idx_entries=idx_e, idx_loci_alleles=idx_l, idx_trait=2,
                                                 add_intercept=False)
    keep = [1, 2, 5, 9]  # entries 4 (row 3, NaN) and 6 (row 5, Inf) dropped
    assert entries == [f"entry_{k - 1}" for k in keep]
    assert np.array_equal(X, g.allele_frequencies[np.ix_(np.array(keep) - 1, idx_l - 1)])
    assert np.array_equal(y, ph.phenotypes[np.array(keep) - 1, 1])
    assert loci == [g.loci_alleles[j - 1] for j in idx_l]


def test_extractxyetc_errors():
    g, ph = make_data()
    with pytest.raises(gbm.ArgumentError, match="out of bounds"):
        gbm.extractxyetc(g, ph, idx_entries=[0, 1])
    with pytest.raises(gbm.ArgumentError, match="out of bounds"):
        gbm.extractxyetc(g, ph, idx_loci_alleles=[61])
    ph2 = gbm.Phenomes(list(reversed(ph.entries)), ph.populations, ph.traits, ph.phenotypes)
    with pytest.raises(gbm.ArgumentError, match="merged"):
        gbm.extractxyetc(g, ph2)
    ph.phenotypes[:, 0] = np.nan
    ph.phenotypes[0, 0] = 1.0
    with pytest.raises(gbm.ArgumentError, match="less than 2"):
        gbm.extractxyetc(g, ph)
    ph.phenotypes[:, 0] = 3.0
    with pytest.raises(gbm.GBMError, match="variance"):
        gbm.extractxyetc(g, ph)
    bad = gbm.Genomes(g.entries[:-1], g.populations, g.loci_alleles, g.allele_frequencies)
    with pytest.raises(gbm.ArgumentError, match="corrupted"):
        gbm.extractxyetc(bad, ph)


def test_predict_checks_before_gpu():
    g, ph = make_data()
    fit = gbm.Fit(n=40, l=61, model="gblup", b_hat_labels=["intercept"] + g.loci_alleles, b_hat=np.zeros(61),
                  entries=g.entries, populations=g.populations)
    assert fit.checkdims()
    with pytest.raises(gbm.ArgumentError, match="out of bounds"):
        gbm.predict(fit, g, [0])
    fit_bad = gbm.Fit(n=40, l=61, model="gblup", b_hat_labels=["intercept"] + ["nope"] * 60, b_hat=np.zeros(61),
                      entries=g.entries, populations=g.populations)
    with pytest.raises(gbm.ArgumentError, match="do not match"):
        gbm.predict(fit_bad, g, [1, 2])
    fit.model = "mystery"
    with pytest.raises(gbm.ArgumentError, match="Unrecognised"):
        gbm.predict(fit, g, [1, 2])
    assert "gblup" in gbm.LINEAR_MODELS and "ridge" in gbm.LINEAR_MODELS


def test_fit_checkdims():
    f = gbm.Fit(n=3, l=5)
    assert f.checkdims()
    f.b_hat = np.zeros(4)
    assert not f.checkdims()


def test_metrics_match_restatement_and_known_values():
    rng = np.random.default_rng(2)
    y = rng.standard_normal(50)
    yp = y + 0.3 * rng.standard_normal(50)
    a, b = gbm.metrics(y, yp), oracle.metrics(y, yp)
    assert set(a) == {"cor", "mad", "msd", "rmsd", "nrmsd", "euc", "jac", "tvar", "h²", "r²"}
    for k in a:
        assert abs(a[k] - b[k]) < 1e-14 * max(1.0, abs(b[k])), k
    assert abs(a["cor"] - np.corrcoef(y, yp)[0, 1]) < 1e-12
    perfect = gbm.metrics(y, y)
    assert perfect["cor"] == pytest.approx(1.0) and perfect["msd"] == 0.0 and perfect["tvar"] == 0.0
    flat = gbm.metrics(y, np.ones(50))  # var(y_pred) < 1e-10 -> 0.0 guards (src/metrics.jl:24-26)
    assert flat["cor"] == 0.0 and flat["r²"] == 0.0 and flat["h²"] == 0.0
