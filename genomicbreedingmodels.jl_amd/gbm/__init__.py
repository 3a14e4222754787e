"""gbm — host-side mirror of GenomicBreedingModels.jl's GBLUP path on MI355X.

Public API mirrors the reference's model-function interface (src/GenomicBreedingModels.jl:35-48):
``extractxyetc``, ``gblup`` (new, beside ``ridge``), ``predict``, ``metrics`` and the data types.
The numerics run in libgbm.so (HIP, gfx950); nothing here falls back to a CPU path.
"""
from ._lib import ArgumentError, GBMError, device_count, load as load_library
from .linear import gblup, gblup_arrays, gblup_dosage, gblup_reml_arrays, gblup_synthetic, glmnet_folds, ridge, ridge_path_cv, ridge_select
from .metrics import heritabilitynarrow_sense, metrics, pearsonscorrelation, r2
from .prediction import LINEAR_MODELS, extractxyetc, predict
from .types import Fit, Genomes, Phenomes
from .arrays import colstats, grm, grm_ploidy_aware, infer_ploidy
from .session import GenotypeSession
from .bayes import bayesian, brr_arrays
from .cv import CV, cvbulk, cvbulk_setup, cvmultithread, fold_assignments, validate

__all__ = [
    "ArgumentError", "GBMError", "device_count", "load_library",
    "gblup", "gblup_arrays", "gblup_dosage", "gblup_reml_arrays", "gblup_synthetic", "ridge", "ridge_path_cv", "ridge_select", "glmnet_folds", "metrics", "pearsonscorrelation", "r2", "heritabilitynarrow_sense",
    "LINEAR_MODELS", "extractxyetc", "predict", "Fit", "Genomes", "Phenomes", "colstats", "grm", "grm_ploidy_aware", "infer_ploidy",
    "GenotypeSession", "bayesian", "brr_arrays", "CV", "cvbulk", "cvbulk_setup", "cvmultithread", "fold_assignments", "validate",
]
