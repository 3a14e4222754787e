"""Bayesian ridge regression (BGLR "BRR") Gibbs sampler — SURVEY.md §8f row 3 (config C4).
BGLR is un-vendored and stochastic: parity vs BGLR itself is unpinned. Pinned instead: the device
sampler (blocked, Gram-based) against the oracle's literal single-site BGLR loop on the same
counter-based random numbers (same sample path), plus distributional checks (posterior-mean GEBVs
vs GBLUP at the matching λ; the reference doctest's cor > 0.5, src/bayes.jl:155-158)."""
import numpy as np
import pytest

import gbm
import oracle


def test_oracle_rng_properties():
    z = np.array([oracle.brr_normal(7, 3, k) for k in range(4000)])
    assert abs(z.mean()) < 0.06 and abs(z.std() - 1) < 0.05
    c = np.array([oracle.brr_chisq(7, k, 9.0) for k in range(2000)])
    assert abs(c.mean() - 9.0) < 0.3 and abs(c.var() - 18.0) < 2.5


def test_oracle_brr_shrinks_like_ridge():
    X = oracle.synth_genotypes(51, 120, 200)
    y = oracle.synth_phenotypes(X, 52)[:, 0]
    r = oracle.brr_gibbs(X, y, n_iter=150, n_burnin=50, thin=5, seed=1)
    assert np.corrcoef(r["y_pred"], y)[0, 1] > 0.5


@pytest.mark.gpu
@pytest.mark.parametrize("n,p,iters", [(100, 300, 12), (77, 130, 9), (200, 64, 7)])
def test_gpu_brr_same_sample_path_as_oracle(n, p, iters):
    X = oracle.synth_genotypes(61 + p, n, p)
    y = oracle.synth_phenotypes(X, 62)[:, 0]
    ref = oracle.brr_gibbs(X, y, n_iter=iters, n_burnin=2, thin=1, seed=99)
    b_hat, y_pred, var = gbm.brr_arrays(X, y, n_iter=iters, n_burnin=2, thin=1, seed=99)
    rel = lambda a, b: np.abs(a - b).max() / np.abs(b).max()
    assert rel(b_hat, ref["b_hat"]) < 1e-9
    assert rel(y_pred, ref["y_pred"]) < 1e-9
    assert abs(var[0] - ref["varE"]) < 1e-9 * ref["varE"] and abs(var[1] - ref["varB"]) < 1e-9 * ref["varB"]


@pytest.mark.gpu
def test_gpu_brr_multi_chunk_matches_oracle():
    """n = 1100: five 256-individual chunks, the partial-dot reduction across workgroups."""
    X = oracle.synth_genotypes(91, 1100, 300)
    y = oracle.synth_phenotypes(X, 92)[:, 0]
    ref = oracle.brr_gibbs(X, y, n_iter=6, n_burnin=2, thin=1, seed=5)
    b_hat, y_pred, var = gbm.brr_arrays(X, y, n_iter=6, n_burnin=2, thin=1, seed=5)
    rel = lambda a, b: np.abs(a - b).max() / np.abs(b).max()
    assert rel(b_hat, ref["b_hat"]) < 1e-9 and rel(y_pred, ref["y_pred"]) < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("n,p", [(700, 450), (1100, 129), (300, 128), (513, 1000)])
def test_gpu_brr_byte_storage_matches_fp64_and_oracle(gbm_env, n, p):
    """Allele frequencies k/2 are stored as bytes for the sweeps (x = d/2 exactly) and run in
    128-marker blocks (two 64-marker halves: δ_A = M_A r̃_A, δ_B = M_B r̃_B + O r̃_A) inside one
    persistent sweep launch; the fp64 storage (GBM_BRR_I8=0) runs one launch per 64-marker block. Same sample path: both agree with each
    other and with the oracle's literal loop to rounding (ragged last blocks: p mod 128 = 66, 1,
    0, 104)."""
    X = oracle.synth_genotypes(93 + p, n, p)
    y = oracle.synth_phenotypes(X, 94)[:, 0]
    got = gbm.brr_arrays(X, y, n_iter=8, n_burnin=2, thin=1, seed=11)
    gbm_env.setenv("GBM_BRR_I8", "0")
    f64 = gbm.brr_arrays(X, y, n_iter=8, n_burnin=2, thin=1, seed=11)
    ref = oracle.brr_gibbs(X, y, n_iter=8, n_burnin=2, thin=1, seed=11)
    rel = lambda a, b: np.abs(a - b).max() / np.abs(b).max()
    for a, b in zip(got, f64):
        assert rel(a, b) < 1e-10
    assert rel(got[0], ref["b_hat"]) < 1e-9 and rel(got[1], ref["y_pred"]) < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("n,p", [(1100, 300), (12000, 260)])
def test_gpu_brr_sweep_matches_per_launch_path_and_oracle(gbm_env, n, p):
    """Byte storage: the persistent super-block sweep (one launch per iteration, hand-offs between
    the chunk workgroups through self-validating write-through granules) against one launch per
    128-marker block (GBM_BRR_SWEEP=0) and the oracle's literal loop. n = 12 000: 250 chunk
    workgroups of 48 individuals, near the sweep's limit."""
    X = oracle.synth_genotypes(97 + n, n, p)
    y = oracle.synth_phenotypes(X, 98)[:, 0]
    _, fb0 = brr_path()
    sweep = gbm.brr_arrays(X, y, n_iter=5, n_burnin=1, thin=1, seed=17)
    assert brr_path() == (4, fb0)
    gbm_env.setenv("GBM_BRR_SWEEP", "0")
    launches = gbm.brr_arrays(X, y, n_iter=5, n_burnin=1, thin=1, seed=17)
    ref = oracle.brr_gibbs(X, y, n_iter=5, n_burnin=1, thin=1, seed=17)
    rel = lambda a, b: np.abs(a - b).max() / np.abs(b).max()
    for a, b in zip(sweep, launches):
        assert rel(a, b) < 1e-11
    assert rel(sweep[0], ref["b_hat"]) < 1e-9 and rel(sweep[1], ref["y_pred"]) < 1e-9


@pytest.mark.gpu
def test_gpu_brr_non_dyadic_genotypes_use_fp64_storage():
    """Values that are not k/s (s = 2, 4, 1) keep fp64 storage; the chain still follows the oracle."""
    X = oracle.synth_genotypes(95, 300, 200) * 0.3 + 0.05
    y = oracle.synth_phenotypes(X, 96)[:, 0]
    ref = oracle.brr_gibbs(X, y, n_iter=6, n_burnin=2, thin=1, seed=13)
    b_hat, y_pred, var = gbm.brr_arrays(X, y, n_iter=6, n_burnin=2, thin=1, seed=13)
    rel = lambda a, b: np.abs(a - b).max() / np.abs(b).max()
    assert rel(b_hat, ref["b_hat"]) < 1e-9 and rel(y_pred, ref["y_pred"]) < 1e-9


@pytest.mark.gpu
def test_gpu_brr_posterior_mean_close_to_gblup():
    """With σ²_b, σ²_e near their posterior the BRR posterior mean of Xb is the ridge/GBLUP BLUP:
    compare GEBVs with GBLUP at λ = σ²_e/σ²_b (posterior means) — distributional, not exact."""
    X = oracle.synth_genotypes(71, 400, 2000)
    y = oracle.synth_phenotypes(X, 72)[:, 0]
    b_hat, y_pred, var = gbm.brr_arrays(X, y, n_iter=1500, n_burnin=500, thin=5, seed=3)
    lam_rr = var[0] / var[1]  # per-marker ridge λ on unscaled X
    # ridge_exact takes glmnet's λ, whose penalty is nλ/σ_y (σ_y = population sd of y)
    a0, b = oracle.ridge_exact(X, y, lam_rr * y.std() / X.shape[0])
    ridge_pred = a0 + X @ b
    assert np.corrcoef(y_pred, ridge_pred)[0, 1] > 0.98
    assert np.corrcoef(y_pred, y)[0, 1] > 0.5


@pytest.mark.gpu
def test_gpu_bayesian_model_function():
    X = oracle.synth_genotypes(81, 150, 500)
    Y = oracle.synth_phenotypes(X, 82)
    ent = [f"e{i}" for i in range(150)]
    g = gbm.Genomes(ent, ["p"] * 150, [f"l{j}" for j in range(500)], X)
    ph = gbm.Phenomes(ent, ["p"] * 150, ["t"], Y)
    fit = gbm.bayesian("BRR", genomes=g, phenomes=ph, n_iter=300, n_burnin=100)
    assert fit.model == "BRR" and fit.checkdims() and fit.metrics["cor"] > 0.5
    pred = gbm.predict(fit, g, list(range(1, 151)))
    assert np.abs(pred - fit.y_pred).max() < 1e-9 * np.abs(fit.y_pred).max()
    with pytest.raises(gbm.ArgumentError):
        gbm.bayesian("BayesA", genomes=g, phenomes=ph)


@pytest.mark.gpu
@pytest.mark.parametrize("sweep", ["1", "0"])
def test_gpu_brr_pooled_no_allocation_after_warmup_and_threads(gbm_env, sweep):
    """gbm_brr_fit leases a pooled per-device context (VERDICT r02 Weak #9): after a warm-up fit, a
    fit of the same shape makes no device allocation and reuses its captured iteration graph
    (bit-identical results). Four threads fitting at once on one device (cvmultithread! with
    bayesian("BRR")) give the serial results bit for bit: their persistent sweeps take turns
    (a per-device lock), so none can be partly resident and spin on another."""
    import threading
    gbm_env.setenv("GBM_BRR_SWEEP", sweep)
    lib = gbm.load_library()
    X = oracle.synth_genotypes(301, 700, 900)
    ys = [oracle.synth_phenotypes(X, 302 + k)[:, 0] for k in range(4)]
    first = gbm.brr_arrays(X, ys[0], n_iter=6, n_burnin=2, thin=1, seed=5)
    a0 = lib.gbm_device_allocations()
    again = gbm.brr_arrays(X, ys[0], n_iter=6, n_burnin=2, thin=1, seed=5)
    assert lib.gbm_device_allocations() == a0
    for a, b in zip(first, again):
        assert np.array_equal(a, b)
    serial = [gbm.brr_arrays(X, y, n_iter=6, n_burnin=2, thin=1, seed=5) for y in ys]
    out, errs = [None] * 4, []

    def run(k):
        try:
            out[k] = gbm.brr_arrays(X, ys[k], n_iter=6, n_burnin=2, thin=1, seed=5)
        except Exception as e:  # reported below
            errs.append(repr(e))

    th = [threading.Thread(target=run, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for a, b in zip(out, serial):
        for u, v in zip(a, b):
            assert np.array_equal(u, v)


def brr_path():
    import ctypes
    lib = gbm.load_library()
    path, fb = ctypes.c_int(-1), ctypes.c_int64(0)
    lib.gbm_debug_brr_stats(ctypes.byref(path), ctypes.byref(fb))
    return path.value, fb.value


@pytest.mark.gpu
@pytest.mark.parametrize("n,p,K", [(1100, 300, None), (12000, 1300, None), (5000, 777, "48"), (3000, 1025, "32"),
                                   (10000, 1100, None), (4000, 900, None), (6000, 2600, None), (10000, 1100, "R4"),
                                   (9000, 2100, "R2")])
def test_gpu_brr_super_block_sweep_runs_and_matches(gbm_env, n, p, K):
    """The super-block sweep really runs (no fall-back to the per-launch path): chunks of <= 48
    individuals, two granule hand-offs per super-block, two steps of slack for the partial dots
    (brr_sweep_la2_kernel, path 4: C2_s δ_{s−2} + C_s δ_{s−1} on the chain). It agrees with the
    per-launch path and the oracle's literal loop; ragged p (p mod 512 = 300, 276, 265, 1, 76)
    including nsb = 1, 2, 3, 6; several chunk sizes, and the owner/non-owner chunk split (owners of
    R = 4, 2 rows with smaller chunks). (The round-3 schedules 1-3 are no longer built.)"""
    if K and K.startswith("R"):  # owners of R rows in the chunk split
        gbm_env.setenv("GBM_BRR_OWN_R", K[1:])
    elif K:
        gbm_env.setenv("GBM_BRR_SB_K", K)
    X = oracle.synth_genotypes(n + p, n, p)
    y = oracle.synth_phenotypes(X, 17)[:, 0]
    _, fb0 = brr_path()
    la2 = gbm.brr_arrays(X, y, n_iter=4, n_burnin=1, thin=1, seed=23)
    path, fb = brr_path()
    assert path == 4 and fb == fb0
    gbm_env.setenv("GBM_BRR_SWEEP", "0")
    launches = gbm.brr_arrays(X, y, n_iter=4, n_burnin=1, thin=1, seed=23)
    assert brr_path()[0] == 0
    rel = lambda a, b: np.abs(a - b).max() / np.abs(b).max()
    for e, c in zip(la2, launches):
        assert rel(e, c) < 1e-10
    if n * p <= 5000 * 1000:
        ref = oracle.brr_gibbs(X, y, n_iter=4, n_burnin=1, thin=1, seed=23)
        assert rel(la2[0], ref["b_hat"]) < 1e-9 and rel(la2[1], ref["y_pred"]) < 1e-9


@pytest.mark.gpu
def test_gpu_brr_fallback_is_reported(gbm_env):
    """A sweep whose hand-offs time out is re-run on the per-launch path; the call succeeds (valid
    results, equal to the per-launch fit) but says so: gbm_last_error() starts with "warning", the
    Python mirror raises a RuntimeWarning, the fall-back counter grows. GBM_BRR_TEST_SWEEP_TIMEOUT
    makes the host treat a completed sweep as timed out (no device-side timeout is provoked)."""
    X = oracle.synth_genotypes(55, 1200, 700)
    y = oracle.synth_phenotypes(X, 56)[:, 0]
    gbm_env.setenv("GBM_BRR_SWEEP", "0")
    ref = gbm.brr_arrays(X, y, n_iter=4, n_burnin=1, thin=1, seed=9)
    gbm_env.delenv("GBM_BRR_SWEEP")
    gbm.brr_arrays(X, y, n_iter=4, n_burnin=1, thin=1, seed=9)
    assert gbm._lib.last_error() == ""  # a clean sweep fit leaves no message
    _, fb0 = brr_path()
    gbm_env.setenv("GBM_BRR_TEST_SWEEP_TIMEOUT", "1")
    with pytest.warns(RuntimeWarning, match="per-launch path"):
        got = gbm.brr_arrays(X, y, n_iter=4, n_burnin=1, thin=1, seed=9)
    assert brr_path() == (0, fb0 + 1)
    assert gbm._lib.last_error().startswith("warning")
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)
