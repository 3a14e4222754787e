"""Array-level wrappers of the GRM and column-statistics entry points (gbm_grm, gbm_colstats)."""
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
