"""Array-level wrappers of the GRM and column-statistics entry points (gbm_grm, gbm_grm_ploidy_aware,
gbm_colstats)."""
from __future__ import annotations

import numpy as np

from . import _lib


def grm(X: np.ndarray, devices=None):
    """G = Z Zᵀ / q on the GPU (replaces Core's grmsimple, reference src/gwas.jl:124). Returns (G, q)."""
    X = np.asfortranarray(np.asarray(X, dtype=np.float64))
    n, p = X.shape
    G = np.zeros((n, n), order="F")
    q = np.zeros(1, dtype=np.int64)
    devs, ndev = _lib.devices_arg(devices)
    rc = _lib.load().gbm_grm(_lib.ptr(X), n, p, n, devs, ndev, _lib.ptr(G), n, _lib.ptr(q))
    _lib.check(rc, "gbm_grm")
    return G, int(q[0])


def infer_ploidy(X: np.ndarray) -> int:
    """The reference's ploidy inference for the ploidy-aware GRM: round(1 / smallest non-zero
    allele frequency) (src/gwas.jl:119)."""
    X = np.asarray(X, dtype=np.float64)
    nz = X[X != 0.0]
    if nz.size == 0:
        raise ValueError("no non-zero allele frequency to infer the ploidy from")
    return int(round(1.0 / nz.min()))


def grm_ploidy_aware(X: np.ndarray, ploidy: int | None = None, devices=None):
    """Ploidy-aware GRM on the GPU (replaces Core's grmploidyaware, reference src/gwas.jl:117-121;
    ploidy inferred as the reference does when None). G = k (X − 1fᵀ)(X − 1fᵀ)ᵀ / Σ f(1 − f), f the
    column means (VanRaden 2008 for ploidy k; the Core formula is un-vendored: parity unpinned).
    Returns (G, Σ f(1 − f))."""
    X = np.asfortranarray(np.asarray(X, dtype=np.float64))
    n, p = X.shape
    k = infer_ploidy(X) if ploidy is None else int(ploidy)
    G = np.zeros((n, n), order="F")
    den = np.zeros(1)
    devs, ndev = _lib.devices_arg(devices)
    rc = _lib.load().gbm_grm_ploidy_aware(_lib.ptr(X), n, p, n, k, devs, ndev, _lib.ptr(G), n, _lib.ptr(den))
    _lib.check(rc, "gbm_grm_ploidy_aware")
    return G, float(den[0])


def colstats(X: np.ndarray, device: int = 0):
    """mean, std (ddof=1), keep mask, q (reference src/gwas.jl:112-113) on the GPU."""
    X = np.asfortranarray(np.asarray(X, dtype=np.float64))
    n, p = X.shape
    m = np.zeros(p)
    s = np.zeros(p)
    k = np.zeros(p, dtype=np.uint8)
    q = np.zeros(1, dtype=np.int64)
    rc = _lib.load().gbm_colstats(_lib.ptr(X), n, p, n, device, _lib.ptr(m), _lib.ptr(s), _lib.ptr(k), _lib.ptr(q))
    _lib.check(rc, "gbm_colstats")
    return m, s, k.astype(bool), int(q[0])
