"""``bayesian`` — mirror of reference src/bayes.jl:158-224 for ``bglr_model = "BRR"`` (Bayesian
ridge regression), with the Gibbs sampler on the GPU (libgbm ``gbm_brr_fit``) instead of an
Rscript/BGLR round trip (src/bayes.jl:28-105). SURVEY.md §8f row 3, config C4."""
from __future__ import annotations

import warnings

import numpy as np

from . import _lib
from ._lib import ArgumentError, GBMError
from .metrics import metrics
from .prediction import extractxyetc
from .types import Fit, Genomes, Phenomes

SUPPORTED = ("BRR",)


def brr_arrays(X: np.ndarray, y: np.ndarray, *, n_iter: int = 1500, n_burnin: int = 500, thin: int = 5,
               r2: float = 0.5, df0: float = 5.0, seed: int = 42, device: int = 0):
    """Array-level BRR Gibbs sampler. Returns (b_hat (p+1,), y_pred (n,), [σ²_e, σ²_b] posterior means)."""
    X = np.asfortranarray(np.asarray(X, dtype=np.float64))
    y = np.ascontiguousarray(np.asarray(y, dtype=np.float64))
    n, p = X.shape
    b_hat = np.zeros(p + 1)
    y_pred = np.zeros(n)
    var = np.zeros(2)
    lib = _lib.load()
    rc = lib.gbm_brr_fit(_lib.ptr(X), n, p, n, _lib.ptr(y), int(n_iter), int(n_burnin), int(thin), float(r2),
                         float(df0), int(seed) & 0xFFFFFFFFFFFFFFFF, int(device), _lib.ptr(b_hat), _lib.ptr(y_pred),
                         _lib.ptr(var))
    _lib.check(rc, "gbm_brr_fit")
    msg = _lib.last_error()
    if msg.startswith("warning"):  # the sweep timed out and the fit was re-run on the per-launch path
        warnings.warn(msg, RuntimeWarning, stacklevel=2)
    return b_hat, y_pred, var


def bayesian(bglr_model: str = "BRR", *, genomes: Genomes, phenomes: Phenomes, idx_entries=None,
             idx_loci_alleles=None, idx_trait: int = 1, response_type: str = "gaussian", n_burnin: int = 500,
             n_iter: int = 1500, verbose: bool = False, thin: int = 5, seed: int = 42, device: int = 0) -> Fit:
    """Bayesian genomic prediction, same signature and Fit assembly as the reference
    (src/bayes.jl:158-224). Only the Gaussian BRR model runs here."""
    if bglr_model not in SUPPORTED:
        raise ArgumentError(f"bglr_model `{bglr_model}` is not available on the GPU path; supported: {SUPPORTED}")
    if response_type != "gaussian":
        raise ArgumentError("only response_type = 'gaussian' is supported")
    X, y, entries, populations, loci_alleles = extractxyetc(
        genomes, phenomes, idx_entries=idx_entries, idx_loci_alleles=idx_loci_alleles, idx_trait=idx_trait,
        add_intercept=False)
    fit = Fit(n=X.shape[0], l=X.shape[1] + 1)
    fit.model = bglr_model
    fit.b_hat_labels = ["intercept"] + list(loci_alleles)
    fit.trait = phenomes.traits[idx_trait - 1]
    fit.entries = entries
    fit.populations = populations
    fit.y_true = y
    b_hat, y_pred, var = brr_arrays(X, y, n_iter=n_iter, n_burnin=n_burnin, thin=thin, seed=seed, device=device)
    fit.b_hat = b_hat
    fit.y_pred = y_pred
    fit.metrics = metrics(y, y_pred)
    if verbose:
        print(fit.metrics, "posterior means: varE", var[0], "varB", var[1])
    if not fit.checkdims():
        raise GBMError("Error fitting " + fit.model + ".")
    return fit
