"""``extractxyetc`` and ``predict`` — host mirrors of reference src/prediction.jl.

``extractxyetc`` is data plumbing (CPU, like the reference). ``predict`` computes the
linear predictor of src/prediction.jl:228 on the GPU (``gbm_predict``), with the reference's
argument checks and label lookup.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from ._lib import ArgumentError, GBMError
from .types import Fit, Genomes, Phenomes

# src/prediction.jl:225 plus the new "gblup" (SURVEY.md §8b decision)
LINEAR_MODELS = ("ols", "ridge", "lasso", "bayesa", "bayesb", "bayesc", "gblup", "BRR")


def extractxyetc(genomes: Genomes, phenomes: Phenomes, idx_entries=None, idx_loci_alleles=None,
                 idx_trait: int = 1, add_intercept: bool = True):
    """Mirror of src/prediction.jl:53-139. Indices are 1-based like Julia's.

    Returns (X, y, entries, populations, loci_alleles) with X Fortran-ordered (column-major,
    as Julia hands it to ``ccall``)."""
    if not genomes.checkdims() and not phenomes.checkdims():
        raise ArgumentError("The Genomes and Phenomes structs are corrupted ☹.")
    if not genomes.checkdims():
        raise ArgumentError("The Genomes struct is corrupted ☹.")
    if not phenomes.checkdims():
        raise ArgumentError("The Phenomes struct is corrupted ☹.")
    if list(genomes.entries) != list(phenomes.entries):
        raise ArgumentError("The genomes and phenomes input need to have been merged to have consitent entries.")
    n_all = len(genomes.entries)
    p_all = len(genomes.loci_alleles)
    if idx_entries is None:
        idx_entries = np.arange(1, n_all + 1)
    else:
        idx_entries = np.asarray(idx_entries, dtype=np.int64)
        if idx_entries.size == 0 or idx_entries.min() < 1 or idx_entries.max() > n_all:
            raise ArgumentError(
                "The indexes of the entries, `idx_entries` are out of bounds. Expected range: from 1 to "
                f"{n_all} while the supplied range is from {idx_entries.min() if idx_entries.size else None} to "
                f"{idx_entries.max() if idx_entries.size else None}.")
    if idx_loci_alleles is None:
        idx_loci_alleles = np.arange(1, p_all + 1)
    else:
        idx_loci_alleles = np.asarray(idx_loci_alleles, dtype=np.int64)
        if idx_loci_alleles.size == 0 or idx_loci_alleles.min() < 1 or idx_loci_alleles.max() > p_all:
            raise ArgumentError(
                "The indexes of the loci_alleles, `idx_loci_alleles` are out of bounds. Expected range: from 1 to "
                f"{p_all} while the supplied range is from "
                f"{idx_loci_alleles.min() if idx_loci_alleles.size else None} to "
                f"{idx_loci_alleles.max() if idx_loci_alleles.size else None}.")
    if not (1 <= idx_trait <= len(phenomes.traits)):
        raise ArgumentError(f"idx_trait = {idx_trait} is out of bounds (1 to {len(phenomes.traits)}).")
    phi = np.asarray(phenomes.phenotypes[idx_entries - 1, idx_trait - 1], dtype=np.float64)
    idx = np.nonzero(np.isfinite(phi))[0]  # drops missing (NaN) and ±Inf, src/prediction.jl:116
    if idx.size < 2:
        raise ArgumentError(
            "There are less than 2 entries with non-missing phenotype data after merging with the genotype data.")
    y = phi[idx]
    if y.var(ddof=1) < 1e-20:
        raise GBMError("Very low or zero variance in trait: `" + str(phenomes.traits[idx_trait - 1]) + "`.")
    rows = idx_entries[idx] - 1
    cols = idx_loci_alleles - 1
    G = np.asfortranarray(np.asarray(genomes.allele_frequencies, dtype=np.float64)[np.ix_(rows, cols)])
    entries = [genomes.entries[r] for r in rows]
    populations = [genomes.populations[r] for r in rows]
    loci_alleles = [genomes.loci_alleles[c] for c in cols]
    if add_intercept:
        return np.asfortranarray(np.hstack([np.ones((idx.size, 1)), G])), y, entries, populations, loci_alleles
    return G, y, entries, populations, loci_alleles


def predict(fit: Fit, genomes: Genomes, idx_entries, device: int = 0) -> np.ndarray:
    """Mirror of src/prediction.jl:189-235; the GEMV ``b_hat[1] .+ X*b_hat[2:end]`` runs on the GPU."""
    if not fit.checkdims():
        raise ArgumentError("The Fit struct is corrupted ☹.")
    if not genomes.checkdims():
        raise ArgumentError("The Genomes struct is corrupted ☹.")
    idx_entries = np.asarray(idx_entries, dtype=np.int64)
    n_all = len(genomes.entries)
    if idx_entries.size == 0 or idx_entries.min() < 1 or idx_entries.max() > n_all:
        raise ArgumentError(
            "The indexes of the entries, `idx_entries` are out of bounds. Expected range: from 1 to "
            f"{n_all} while the supplied range is from {idx_entries.min() if idx_entries.size else None} to "
            f"{idx_entries.max() if idx_entries.size else None}.")
    # label lookup (src/prediction.jl:215-223); a dict instead of the O(p²) findall
    pos = {lab: k for k, lab in enumerate(genomes.loci_alleles)}
    try:
        idx_loci = np.array([pos[lab] for lab in fit.b_hat_labels[1:]], dtype=np.int64)
    except KeyError:
        raise ArgumentError(
            "The loci-alleles in the fitted genomic prediction model do not match the loci-alleles in the "
            "requested validation set.") from None
    if fit.model in LINEAR_MODELS:
        X = np.asfortranarray(np.asarray(genomes.allele_frequencies, dtype=np.float64)[np.ix_(idx_entries - 1, idx_loci)])
        b = np.ascontiguousarray(np.asarray(fit.b_hat, dtype=np.float64))
        n, p = X.shape
        out = np.empty(n)
        lib = _lib.load()
        rc = lib.gbm_predict(_lib.ptr(X), n, p, n, _lib.ptr(b), p + 1, 1, device, _lib.ptr(out), n)
        _lib.check(rc, "gbm_predict")
        return out
    raise ArgumentError("Unrecognised genomic prediction model: `" + fit.model + "`.")
