"""Device-resident genotype sessions (libgbm ``gbm_session_*``): the fold-farming runtime behind
``cvmultithread``/``cvbulk`` and the REML choice of λ (row 2).

X is uploaded once per device; each fit gathers its training rows on the device, and the
standardised training genotypes + GRM are cached per training set (reference
src/cross_validation.jl:159-186 refits everything per fold)."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import ArgumentError


def _idx(idx) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(idx, dtype=np.int64))
    if a.ndim != 1 or a.size == 0:
        raise ArgumentError("entry indices must be a non-empty 1-D array")
    return a


class GenotypeSession:
    """X (n entries x p loci-alleles, allele frequencies) resident on one device."""

    def __init__(self, X: np.ndarray | None = None, *, device: int = 0, dosage_i8: np.ndarray | None = None,
                 ploidy: int | None = None):
        self.lib = _lib.load()
        self._h = ctypes.c_void_p()
        self.device = int(device)
        if dosage_i8 is not None:
            D = np.asfortranarray(np.asarray(dosage_i8, dtype=np.int8))
            self.n, self.p = D.shape
            if not ploidy or ploidy < 1:
                raise ArgumentError("ploidy must be >= 1 with int8 dosages")
            rc = self.lib.gbm_session_create_dosage_i8(_lib.ptr(D), self.n, self.p, self.n, int(ploidy), self.device,
                                                       ctypes.byref(self._h))
            _lib.check(rc, "gbm_session_create_dosage_i8")
        else:
            X = np.asfortranarray(np.asarray(X, dtype=np.float64))
            if X.ndim != 2:
                raise ArgumentError("X must be a 2-D (entries x loci-alleles) array")
            if not np.isfinite(X).all():
                raise ArgumentError("X has missing/NaN/Inf allele frequencies")
            self.n, self.p = X.shape
            rc = self.lib.gbm_session_create(_lib.ptr(X), self.n, self.p, self.n, self.device, ctypes.byref(self._h))
            _lib.check(rc, "gbm_session_create")

    @classmethod
    def synthetic(cls, seed: int, n: int, p: int, *, device: int = 0) -> "GenotypeSession":
        """Session over the counter-hash synthetic genotypes of loci 0..p-1, generated
        on the device (benchmark-scale configs without a host copy of X)."""
        self = cls.__new__(cls)
        self.lib = _lib.load()
        self._h = ctypes.c_void_p()
        self.device = int(device)
        self.n, self.p = int(n), int(p)
        _lib.check(self.lib.gbm_session_create_synthetic(int(seed), self.n, self.p, self.device, ctypes.byref(self._h)),
                   "gbm_session_create_synthetic")
        return self

    # ---- lifetime -------------------------------------------------------------------------
    def close(self):
        if self._h:
            self.lib.gbm_session_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover - interpreter teardown order
        try:
            self.close()
        except Exception:
            pass

    # ---- GRM arithmetic -----------------------------------------------------------------------
    def set_grm(self, grm):
        """GRM arithmetic of the training GRMs: None (the GBM_GRM variable, else fp64), "fp64", "exact" or
        "auto" (exact when the genotypes are diploid dosages/2; include/gbm.h gbm_session_set_grm_mode)."""
        _lib.check(self.lib.gbm_session_set_grm_mode(self._h, _lib.grm_mode(grm)), "gbm_session_set_grm_mode")
        return self

    def grm_used(self):
        """"fp64" or "exact": the GRM the cached training set was built with (None before the first fit)."""
        v = ctypes.c_int(-1)
        _lib.check(self.lib.gbm_session_grm_used(self._h, ctypes.byref(v)), "gbm_session_grm_used")
        return {_lib.GBM_GRM_FP64: "fp64", _lib.GBM_GRM_EXACT: "exact"}.get(v.value)

    # ---- model calls ----------------------------------------------------------------------
    def gblup(self, idx, Y, lambda_: float = 1.0):
        """GBLUP on rows ``idx`` (0-based, strictly increasing); Y (n_train,) or (n_train, t).
        Returns (b_hat (p+1, t), y_pred (n_train, t), mu (t,), q)."""
        idx = _idx(idx)
        Y = np.asarray(Y, dtype=np.float64)
        if Y.ndim == 1:
            Y = Y[:, None]
        Y = np.asfortranarray(Y)
        m, t = Y.shape
        if m != idx.size:
            raise ArgumentError("Y rows must match the training indices")
        b_hat = np.zeros((self.p + 1, t), order="F")
        y_pred = np.zeros((m, t), order="F")
        mu = np.zeros(t)
        q = np.zeros(1, dtype=np.int64)
        rc = self.lib.gbm_session_gblup_fit(self._h, _lib.ptr(idx), m, _lib.ptr(Y), m, t, float(lambda_),
                                            _lib.ptr(b_hat), _lib.ptr(y_pred), _lib.ptr(mu), _lib.ptr(q))
        _lib.check(rc, "gbm_session_gblup_fit")
        return b_hat, y_pred, mu, int(q[0])

    def predict(self, idx, b_hat) -> np.ndarray:
        """b0 + X[idx, :] b for b_hat (p+1,) or (p+1, t); returns (n_val,) or (n_val, t)."""
        idx = _idx(idx)
        b = np.asarray(b_hat, dtype=np.float64)
        one = b.ndim == 1
        if one:
            b = b[:, None]
        b = np.asfortranarray(b)
        if b.shape[0] != self.p + 1:
            raise ArgumentError("b_hat must have p + 1 rows (intercept first)")
        t = b.shape[1]
        out = np.zeros((idx.size, t), order="F")
        rc = self.lib.gbm_session_predict(self._h, _lib.ptr(idx), idx.size, _lib.ptr(b), self.p + 1, t,
                                          _lib.ptr(out), idx.size)
        _lib.check(rc, "gbm_session_predict")
        return out[:, 0].copy() if one else out

    def reml_objective(self, idx, y, sigma2_e, sigma2_u) -> np.ndarray:
        """Reference loglikreml (src/gwas.jl:450-483) with X = 1 at the given (σ²_e, σ²_u) pairs."""
        idx = _idx(idx)
        y = np.ascontiguousarray(np.asarray(y, dtype=np.float64))
        se = np.ascontiguousarray(np.atleast_1d(np.asarray(sigma2_e, dtype=np.float64)))
        su = np.ascontiguousarray(np.atleast_1d(np.asarray(sigma2_u, dtype=np.float64)))
        if se.shape != su.shape or y.shape != (idx.size,):
            raise ArgumentError("shape mismatch")
        out = np.zeros(se.size)
        rc = self.lib.gbm_session_reml_objective(self._h, _lib.ptr(idx), idx.size, _lib.ptr(y), _lib.ptr(se),
                                                 _lib.ptr(su), se.size, _lib.ptr(out))
        _lib.check(rc, "gbm_session_reml_objective")
        return out

    def reml(self, idx, y) -> dict:
        """REML λ = σ²_e/σ²_u for standardised y over the reference's box [eps, 1]² (src/gwas.jl:585)."""
        idx = _idx(idx)
        y = np.ascontiguousarray(np.asarray(y, dtype=np.float64))
        if y.shape != (idx.size,):
            raise ArgumentError("y must have one value per training index")
        v = np.zeros(4)
        p = [ctypes.c_void_p(v.ctypes.data + 8 * k) for k in range(4)]
        rc = self.lib.gbm_session_reml(self._h, _lib.ptr(idx), idx.size, _lib.ptr(y), *p)
        _lib.check(rc, "gbm_session_reml")
        return {"lambda": float(v[0]), "sigma2_e": float(v[1]), "sigma2_u": float(v[2]), "objective": float(v[3])}

    def ridge_lambda_max(self, idx, y) -> float:
        """glmnet's first λ for alpha = 0 on rows ``idx`` (standardize = false)."""
        idx = _idx(idx)
        y = np.ascontiguousarray(np.asarray(y, dtype=np.float64))
        out = np.zeros(1)
        rc = self.lib.gbm_session_ridge_lambda_max(self._h, _lib.ptr(idx), idx.size, _lib.ptr(y), _lib.ptr(out))
        _lib.check(rc, "gbm_session_ridge_lambda_max")
        return float(out[0])

    def ridge_path(self, idx, y, lambdas, idx_eval=None):
        """Exact glmnet ridge solutions (alpha = 0, standardize = false, intercept) on rows ``idx``
        at each λ. Returns b_path (p+1, nl) [intercept first] and, with ``idx_eval``, the
        predictions (n_eval, nl)."""
        idx = _idx(idx)
        y = np.ascontiguousarray(np.asarray(y, dtype=np.float64))
        lam = np.ascontiguousarray(np.atleast_1d(np.asarray(lambdas, dtype=np.float64)))
        b = np.zeros((self.p + 1, lam.size), order="F")
        if idx_eval is not None:
            ie = _idx(idx_eval)
            pred = np.zeros((ie.size, lam.size), order="F")
            rc = self.lib.gbm_session_ridge_path(self._h, _lib.ptr(idx), idx.size, _lib.ptr(y), _lib.ptr(lam),
                                                 lam.size, _lib.ptr(b), _lib.ptr(ie), ie.size, _lib.ptr(pred))
            _lib.check(rc, "gbm_session_ridge_path")
            return b, pred
        rc = self.lib.gbm_session_ridge_path(self._h, _lib.ptr(idx), idx.size, _lib.ptr(y), _lib.ptr(lam), lam.size,
                                             _lib.ptr(b), None, 0, None)
        _lib.check(rc, "gbm_session_ridge_path")
        return b

    def stats(self):
        """(GRM builds, GRM cache hits)."""
        v = np.zeros(2, dtype=np.int64)
        rc = self.lib.gbm_session_stats(self._h, ctypes.c_void_p(v.ctypes.data), ctypes.c_void_p(v.ctypes.data + 8))
        _lib.check(rc, "gbm_session_stats")
        return int(v[0]), int(v[1])
