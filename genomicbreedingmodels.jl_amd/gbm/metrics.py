"""Prediction metrics — mirror of reference src/metrics.jl:23-128 (Distances.jl semantics restated;
``var`` is Julia's sample variance, ddof = 1). CPU-side like the reference (n-vectors)."""
from __future__ import annotations

import numpy as np


def _var(v: np.ndarray) -> float:
    return float(v.var(ddof=1)) if v.size > 1 else float("nan")


def pearsonscorrelation(y_true, y_pred) -> float:
    """src/metrics.jl:23-29: 0.0 when either variance < 1e-10, else 1 − corr_dist."""
    y_true = np.asarray(y_true, dtype=np.float64)
    y_pred = np.asarray(y_pred, dtype=np.float64)
    if _var(y_true) < 1e-10 or _var(y_pred) < 1e-10:
        return 0.0
    a = y_true - y_true.mean()
    b = y_pred - y_pred.mean()
    return float(1.0 - (1.0 - (a @ b) / np.sqrt((a @ a) * (b @ b))))


def r2(y_true, y_pred) -> float:
    """src/metrics.jl:41-49."""
    y_true = np.asarray(y_true, dtype=np.float64)
    y_pred = np.asarray(y_pred, dtype=np.float64)
    if _var(y_true) < 1e-10 or _var(y_pred) < 1e-10:
        return 0.0
    return float(1.0 - _var(y_true - y_pred) / _var(y_true))


def heritabilitynarrow_sense(y_true, y_pred) -> float:
    """src/metrics.jl:73-90 (clamped to [0, 1])."""
    y_true = np.asarray(y_true, dtype=np.float64)
    y_pred = np.asarray(y_pred, dtype=np.float64)
    if _var(y_true) < 1e-10 or _var(y_pred) < 1e-10:
        return 0.0
    s2a = _var(y_pred)
    s2e = _var(y_true - y_pred)
    h2 = s2a / (s2a + s2e) if (s2a + s2e) >= 1e-20 else 0.0
    return float(min(max(h2, 0.0), 1.0))


def metrics(y_true, y_pred) -> dict:
    """src/metrics.jl:115-128: cor, mad, msd, rmsd, nrmsd, euc, jac, tvar, h², r²."""
    y_true = np.asarray(y_true, dtype=np.float64)
    y_pred = np.asarray(y_pred, dtype=np.float64)
    d = y_true - y_pred
    msd = float(np.mean(d * d))
    rmsd = float(np.sqrt(msd))
    return {
        "cor": pearsonscorrelation(y_true, y_pred),
        "mad": float(np.mean(np.abs(d))),                      # Distances.meanad
        "msd": msd,                                           # Distances.msd
        "rmsd": rmsd,                                         # Distances.rmsd
        "nrmsd": float(rmsd / (y_true.max() - y_true.min())),  # rmsd / (max(a) − min(a))
        "euc": float(np.sqrt(np.sum(d * d))),                  # Distances.euclidean
        "jac": float(1.0 - np.sum(np.minimum(y_true, y_pred)) / np.sum(np.maximum(y_true, y_pred))),
        "tvar": float(0.5 * np.sum(np.abs(d))),                 # Distances.totalvariation
        "h²": heritabilitynarrow_sense(y_true, y_pred),
        "r²": r2(y_true, y_pred),
    }
