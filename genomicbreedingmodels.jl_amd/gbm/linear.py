"""``gblup`` model function — the drop-in beside reference ``ridge`` (src/linear.jl:162-239).

Same keyword signature as every reference model function (the six keywords
``cvmultithread!`` passes at src/cross_validation.jl:170-177, plus ``lambda_`` with a default),
same Fit assembly sequence (src/linear.jl:185-191,223-238); where ``ridge`` calls
``GLMNet.glmnetcv`` (src/linear.jl:193-203) this calls ``gbm_gblup_fit`` in libgbm.so
(GRM on fp64 MFMA + blocked Cholesky on the MI355X).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import ArgumentError, GBMError
from .metrics import metrics
from .prediction import extractxyetc
from .types import Fit, Genomes, Phenomes


def _grm_info(info, used):
    if info is not None:
        info["grm_used"] = {_lib.GBM_GRM_FP64: "fp64", _lib.GBM_GRM_EXACT: "exact"}.get(int(used.value), int(used.value))


def gblup_arrays(X: np.ndarray, Y: np.ndarray, lambda_: float = 1.0, devices=None, grm=None, info=None):
    """Array-level GBLUP through the C ABI (gbm_gblup_fit_ex). X (n, p) any order, Y (n,) or (n, t).
    ``grm``: the GRM arithmetic (None: the GBM_GRM variable, else fp64; "fp64"; "exact": diploid dosages/2
    only; "auto": exact when every 2x is 0, 1 or 2, else fp64 — include/gbm.h GBM_GRM_*). ``info`` (a dict,
    optional) receives ``grm_used``.

    Returns (b_hat (p+1, t), y_pred (n, t), mu (t,), q)."""
    X = np.asfortranarray(np.asarray(X, dtype=np.float64))
    Y = np.asarray(Y, dtype=np.float64)
    if Y.ndim == 1:
        Y = Y[:, None]
    Y = np.asfortranarray(Y)
    n, p = X.shape
    t = Y.shape[1]
    b_hat = np.zeros((p + 1, t), order="F")
    y_pred = np.zeros((n, t), order="F")
    mu = np.zeros(t)
    q = np.zeros(1, dtype=np.int64)
    devs, ndev = _lib.devices_arg(devices)
    lib = _lib.load()
    used = ctypes.c_int(-1)
    rc = lib.gbm_gblup_fit_ex(_lib.ptr(X), n, p, n, _lib.ptr(Y), n, t, float(lambda_), devs, ndev, _lib.grm_mode(grm),
                              _lib.ptr(b_hat), _lib.ptr(y_pred), _lib.ptr(mu), _lib.ptr(q), ctypes.byref(used))
    _lib.check(rc, "gbm_gblup_fit")
    _grm_info(info, used)
    return b_hat, y_pred, mu, int(q[0])


def gblup_reml_arrays(X: np.ndarray, Y: np.ndarray, devices=None, grm=None, info=None):
    """Array-level GBLUP with λ chosen per trait by REML through the C ABI (gbm_gblup_fit_reml: the
    reference's loglikreml objective, src/gwas.jl:450-483, on the call's own GRM). Returns
    (b_hat (p+1, t), y_pred (n, t), mu (t,), q, reml) with reml = dict(lambda, sigma2_e, sigma2_u) of
    (t,) arrays."""
    X = np.asfortranarray(np.asarray(X, dtype=np.float64))
    Y = np.asarray(Y, dtype=np.float64)
    if Y.ndim == 1:
        Y = Y[:, None]
    Y = np.asfortranarray(Y)
    n, p = X.shape
    t = Y.shape[1]
    b_hat = np.zeros((p + 1, t), order="F")
    y_pred = np.zeros((n, t), order="F")
    mu = np.zeros(t)
    q = np.zeros(1, dtype=np.int64)
    lam, s2e, s2u = np.zeros(t), np.zeros(t), np.zeros(t)
    devs, ndev = _lib.devices_arg(devices)
    used = ctypes.c_int(-1)
    rc = _lib.load().gbm_gblup_fit_reml_ex(_lib.ptr(X), n, p, n, _lib.ptr(Y), n, t, devs, ndev, _lib.grm_mode(grm),
                                           _lib.ptr(b_hat), _lib.ptr(y_pred), _lib.ptr(mu), _lib.ptr(q), _lib.ptr(lam),
                                           _lib.ptr(s2e), _lib.ptr(s2u), ctypes.byref(used))
    _lib.check(rc, "gbm_gblup_fit_reml")
    _grm_info(info, used)
    return b_hat, y_pred, mu, int(q[0]), {"lambda": lam, "sigma2_e": s2e, "sigma2_u": s2u}


def gblup_dosage(D: np.ndarray, ploidy: int, Y: np.ndarray, lambda_: float = 1.0, devices=None, grm=None, info=None):
    """GBLUP on int8 dosages (gbm_gblup_fit_dosage_i8: X = D/ploidy, 1 byte per cell over PCIe).
    D (n, p) int8, any order. Returns (b_hat (p+1, t), y_pred (n, t), mu (t,), q)."""
    D = np.asfortranarray(np.asarray(D, dtype=np.int8))
    Y = np.asarray(Y, dtype=np.float64)
    if Y.ndim == 1:
        Y = Y[:, None]
    Y = np.asfortranarray(Y)
    n, p = D.shape
    t = Y.shape[1]
    b_hat = np.zeros((p + 1, t), order="F")
    y_pred = np.zeros((n, t), order="F")
    mu = np.zeros(t)
    q = np.zeros(1, dtype=np.int64)
    dev, nd = _lib.devices_arg(devices)
    used = ctypes.c_int(-1)
    _lib.check(_lib.load().gbm_gblup_fit_dosage_i8_ex(_lib.ptr(D), n, p, n, int(ploidy), _lib.ptr(Y), n, t,
                                                     float(lambda_), dev, nd, _lib.grm_mode(grm), _lib.ptr(b_hat),
                                                     _lib.ptr(y_pred), _lib.ptr(mu), _lib.ptr(q), ctypes.byref(used)),
               "gbm_gblup_fit_dosage_i8")
    _grm_info(info, used)
    return b_hat, y_pred, mu, int(q[0])


def gblup_synthetic(seed: int, n: int, p: int, Y: np.ndarray, lambda_: float = 1.0, devices=None, grm=None, info=None):
    """GBLUP on the device-generated synthetic genotypes (gbm_gblup_fit_synthetic: loci 0..p-1 of the
    SURVEY.md §8d generator, no host X). Returns (b_hat (p+1, t), y_pred (n, t), mu (t,), q)."""
    Y = np.asarray(Y, dtype=np.float64)
    if Y.ndim == 1:
        Y = Y[:, None]
    Y = np.asfortranarray(Y)
    if Y.shape[0] != n:
        raise ArgumentError("Y must have n rows")
    t = Y.shape[1]
    b_hat = np.zeros((p + 1, t), order="F")
    y_pred = np.zeros((n, t), order="F")
    mu = np.zeros(t)
    q = np.zeros(1, dtype=np.int64)
    devs, ndev = _lib.devices_arg(devices)
    lib = _lib.load()
    used = ctypes.c_int(-1)
    rc = lib.gbm_gblup_fit_synthetic_ex(int(seed), n, p, _lib.ptr(Y), n, t, float(lambda_), devs, ndev,
                                        _lib.grm_mode(grm), _lib.ptr(b_hat), _lib.ptr(y_pred), _lib.ptr(mu),
                                        _lib.ptr(q), ctypes.byref(used))
    _lib.check(rc, "gbm_gblup_fit_synthetic")
    _grm_info(info, used)
    return b_hat, y_pred, mu, int(q[0])


def gblup(*, genomes: Genomes, phenomes: Phenomes, idx_entries=None, idx_loci_alleles=None,
          idx_trait: int = 1, verbose: bool = False, lambda_: float = 1.0, devices=None,
          model_label: str = "gblup", grm: str = "dropin") -> Fit:
    """GBLUP / RR-BLUP fit returning a ``Fit`` exactly like ``ridge`` does.

    ``model_label="ridge"`` lets the fit flow through an unmodified reference ``predict``
    whitelist (src/prediction.jl:225): GBLUP ≡ RR-BLUP, so the linear predictor is valid.
    ``lambda_="reml"`` chooses λ = σ²_e/σ²_u by REML first (the REML result is kept in
    ``fit.metrics_reml``). ``grm`` (Julia ``grm = :dropin``): "auto" computes the GRM exactly on the int8
    matrix cores when the allele frequencies are diploid dosages/2 (2x ∈ {0, 1, 2} in every cell, checked on
    the device), else with the fp64-MFMA SYRK; "fp64" / "exact" force one; the default "dropin" is the GBM_GRM
    variable when it is set, else "auto" (include/gbm.h GBM_GRM_*). The GRM used is kept in ``fit.grm_used``."""
    X, y, entries, populations, loci_alleles = extractxyetc(
        genomes, phenomes, idx_entries=idx_entries, idx_loci_alleles=idx_loci_alleles,
        idx_trait=idx_trait, add_intercept=False)
    fit = Fit(n=X.shape[0], l=X.shape[1])
    fit.model = model_label
    fit.b_hat_labels = ["intercept"] + list(loci_alleles)
    fit.trait = phenomes.traits[idx_trait - 1]
    fit.entries = entries
    fit.populations = populations
    fit.y_true = y
    info = {}
    if isinstance(lambda_, str):
        # REML choice of λ through the drop-in entry gbm_gblup_fit_reml: one
        # GRM, REML over the reference's loglikreml objective (src/gwas.jl:450-483), then the fit
        if lambda_ != "reml":
            raise ArgumentError(f"lambda_ must be a positive number or \"reml\", got {lambda_!r}")
        b_hat, y_pred, mu, q, r = gblup_reml_arrays(X, y, devices=devices, grm=grm, info=info)
        lambda_ = float(r["lambda"][0])
        fit.metrics_reml = {k: float(v[0]) for k, v in r.items()}
    else:
        b_hat, y_pred, mu, q = gblup_arrays(X, y, lambda_=lambda_, devices=devices, grm=grm, info=info)
    fit.grm_used = info.get("grm_used")
    fit.b_hat = b_hat[:, 0].copy()
    fit.y_pred = y_pred[:, 0].copy()
    fit.metrics = metrics(y, fit.y_pred)
    if verbose:
        print(f"gblup: n={X.shape[0]} p={X.shape[1]} q={q} mu={mu[0]:.6g} lambda={lambda_} grm={fit.grm_used}")
        print(fit.metrics)
    if not fit.checkdims():
        raise GBMError("Error fitting " + fit.model + ".")
    return fit


def glmnet_folds(n: int, nfolds: int, rng) -> np.ndarray:
    """GLMNet.jl glmnetcv's default folds: ``nfolds = min(10, n ÷ 3)`` balanced labels
    ``[repeat(1:nfolds, n ÷ nfolds); 1:(n % nfolds)]`` shuffled (unseeded there; ``rng`` here)."""
    q, r = divmod(n, nfolds)
    f = np.concatenate([np.tile(np.arange(1, nfolds + 1), q), np.arange(1, r + 1)])
    rng.shuffle(f)
    return f


def ridge_path_cv(X: np.ndarray, y: np.ndarray, *, nlambda: int = 100, lambda_min_ratio: float = 0.01,
                  nfolds: int | None = None, seed: int = 42, device: int = 0):
    """``GLMNet.glmnetcv(X, y, alpha=0, standardize=false, nlambda=100, lambda_min_ratio=0.01,
    intercept=true)`` as called by reference ridge (src/linear.jl:193-203), on the GPU: the λ path
    from the full data, every path solved exactly (kernel form, one Cholesky per λ on the cached
    centred-X kernel), k-fold CV mean squared error per λ. Returns dict(lambda, a0, betas (p, nl),
    meanloss)."""
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    n = X.shape[0]
    nf = nfolds if nfolds is not None else min(10, n // 3)
    if nf < 2:
        raise ArgumentError("glmnetcv needs at least 2 folds (n >= 6)")
    from .session import GenotypeSession
    with GenotypeSession(X, device=device) as s:
        idx = np.arange(n)
        lmax = s.ridge_lambda_max(idx, y)
        lam = lmax * lambda_min_ratio ** (np.arange(nlambda) / (nlambda - 1))
        path = s.ridge_path(idx, y, lam)
        folds = glmnet_folds(n, nf, np.random.default_rng(seed))
        loss = np.zeros((nlambda, nf))
        for f in range(1, nf + 1):
            tr, ho = np.flatnonzero(folds != f), np.flatnonzero(folds == f)
            _, pred = s.ridge_path(tr, y[tr], lam, idx_eval=ho)
            loss[:, f - 1] = ((pred - y[ho, None]) ** 2).mean(axis=0)
    return {"lambda": lam, "a0": path[0].copy(), "betas": path[1:].copy(), "meanloss": loss.mean(axis=1)}


def ridge_select(a0: np.ndarray, betas: np.ndarray, meanloss: np.ndarray) -> np.ndarray:
    """The coefficient choice of reference ridge (src/linear.jl:213-223), quirks included: λs
    sorted by CV loss; the intercept taken as ``a0[idx_sort][idx_sort[i]]`` (a double
    permutation) and the first solution whose slopes have variance >= 1e-10 kept."""
    idx_sort = np.argsort(meanloss, kind="stable")
    intercepts = a0[idx_sort]
    nl = betas.shape[1]
    b_hat = np.zeros(betas.shape[0] + 1)
    i = 0
    while np.var(b_hat[1:], ddof=1) < 1e-10 or i == nl - 1:
        if i >= nl:
            break
        b_hat = np.concatenate([[intercepts[idx_sort[i]]], betas[:, idx_sort[i]]])
        i += 1
    return b_hat


def ridge(*, genomes: Genomes, phenomes: Phenomes, idx_entries=None, idx_loci_alleles=None, idx_trait: int = 1,
          verbose: bool = False, seed: int = 42, device: int = 0) -> Fit:
    """Mirror of reference ``ridge`` (src/linear.jl:162-239) with the GLMNet path on the GPU."""
    X, y, entries, populations, loci_alleles = extractxyetc(
        genomes, phenomes, idx_entries=idx_entries, idx_loci_alleles=idx_loci_alleles,
        idx_trait=idx_trait, add_intercept=False)
    fit = Fit(n=X.shape[0], l=X.shape[1])
    fit.model = "ridge"
    fit.b_hat_labels = ["intercept"] + list(loci_alleles)
    fit.trait = phenomes.traits[idx_trait - 1]
    fit.entries = entries
    fit.populations = populations
    fit.y_true = y
    cv = ridge_path_cv(X, y, seed=seed, device=device)
    b_hat = ridge_select(cv["a0"], cv["betas"], cv["meanloss"])
    from .session import GenotypeSession
    with GenotypeSession(X, device=device) as s:
        y_pred = s.predict(np.arange(X.shape[0]), b_hat)
    fit.b_hat = b_hat
    fit.y_pred = y_pred
    fit.metrics = metrics(y, y_pred)
    if verbose:
        print("argmin =", int(np.argmin(cv["meanloss"])) + 1)
        print(fit.metrics)
    if not fit.checkdims():
        raise GBMError("Error fitting " + fit.model + ".")
    return fit
