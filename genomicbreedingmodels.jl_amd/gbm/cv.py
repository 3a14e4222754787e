"""Cross-validation: ``validate``, ``cvmultithread``, ``cvbulk`` — mirrors of reference
src/cross_validation.jl:49-81, 151-207 and 268-401, with the GBLUP fold jobs farmed onto
device-resident genotype sessions (one per GPU, training-set-keyed GRM cache; SURVEY.md §8f
row 1, config C5).

Fold assignment: the reference samples ``StatsBase.sample(rng, 1:n_folds, n, replace=true)`` per
(trait, replication) from Julia's ``Random.seed!(seed)`` stream (src/cross_validation.jl:359), which
numpy cannot reproduce; here the same scheme draws from ``numpy.random.default_rng(seed)``
(fold assignment parity unpinned; each fold's fit and prediction are pinned to the oracle).
"""
from __future__ import annotations

import functools
import threading
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import ArgumentError, GBMError
from .linear import gblup
from .metrics import metrics
from .prediction import predict
from .session import GenotypeSession
from .types import Fit, Genomes, Phenomes


@dataclass
class CV:
    """Mirror of GenomicBreedingCore's ``CV`` (fields as constructed at src/cross_validation.jl:79,385-394)."""
    replication: str
    fold: str
    fit: Fit
    validation_populations: list
    validation_entries: list
    validation_y_true: np.ndarray
    validation_y_pred: np.ndarray
    metrics: dict = field(default_factory=dict)

    def checkdims(self) -> bool:
        m = len(self.validation_entries)
        return (self.fit.checkdims() and len(self.validation_populations) == m
                and len(self.validation_y_true) == m and len(self.validation_y_pred) == m)


def validate(fit: Fit, genomes: Genomes, phenomes: Phenomes, *, idx_validation, replication: str = "",
             fold: str = "", device: int = 0) -> CV:
    """Mirror of src/cross_validation.jl:49-81 (1-based ``idx_validation``)."""
    idx_trait = phenomes.traits.index(fit.trait)
    idx_validation = np.asarray(idx_validation, dtype=np.int64)
    leak = sorted(set(fit.entries) & {phenomes.entries[i - 1] for i in idx_validation})
    if leak:
        raise ArgumentError("Data leakage between training and validation sets, i.e. entries:\n\t‣ " +
                            "\n\t‣ ".join(leak))
    phi = np.asarray(phenomes.phenotypes, dtype=np.float64)[idx_validation - 1, idx_trait]
    keep = np.isfinite(phi)
    idx = idx_validation[keep]
    y_true = phi[keep]
    y_pred = predict(fit, genomes, idx, device=device)
    cv = CV(replication, fold, fit, [phenomes.populations[i - 1] for i in idx], [phenomes.entries[i - 1] for i in idx],
            y_true, y_pred, metrics(y_true, y_pred))
    if not cv.checkdims():
        raise ArgumentError("CV struct is corrupted ☹.")
    return cv


# ---- GBLUP fold jobs on device sessions ----------------------------------------------------------

def _gblup_lambda(model):
    """λ of a gblup model callable (``gblup`` or ``functools.partial(gblup, lambda_=...)``), else None."""
    if model is gblup:
        return 1.0
    if isinstance(model, functools.partial) and model.func is gblup and not model.args:
        kw = dict(model.keywords)
        lam = kw.pop("lambda_", 1.0)
        kw.pop("devices", None)
        if not kw or set(kw) <= {"model_label"}:
            return lam
    return None


def _model_label(model) -> str:
    if isinstance(model, functools.partial):
        return model.keywords.get("model_label", "gblup") if model.func is gblup else str(model.func.__name__)
    return getattr(model, "__name__", str(model))


@dataclass
class _Job:
    i: int                   # position in cvs
    lam: object              # float or "reml"
    idx_train: np.ndarray    # 0-based rows with finite phenotype, strictly increasing (the session's order)
    order: np.ndarray        # caller order of the training rows: rows_caller = idx_train[order]
    idx_val: np.ndarray      # 0-based rows, caller order
    trait: int               # 0-based trait column


def _make_job(i, lam, rows, idx_val, trait, Y) -> _Job:
    """extractxyetc's row handling (src/prediction.jl:114-131) for a fold job: drop training rows
    whose phenotype is missing/NaN/Inf, keep the caller's order for Fit.entries, and give the
    session the same rows sorted (its index sets are strictly increasing)."""
    rows = np.asarray(rows, dtype=np.int64)
    rows = rows[np.isfinite(Y[rows, trait])]
    perm = np.argsort(rows, kind="stable")
    order = np.empty_like(perm)
    order[perm] = np.arange(perm.size)
    return _Job(i, lam, rows[perm], order, np.asarray(idx_val, dtype=np.int64), trait)


def _sorted_predict(session: GenotypeSession, rows: np.ndarray, b_hat: np.ndarray) -> np.ndarray:
    """session.predict on rows in any order (predictions returned in that order)."""
    if rows.size == 0:
        return np.zeros(0)
    perm = np.argsort(rows, kind="stable")
    out = np.empty(rows.size)
    out[perm] = session.predict(rows[perm], b_hat)
    return out


def _run_device_jobs(session: GenotypeSession, jobs, cvs, genomes, phenomes, errors, lock):
    Yall = np.asarray(phenomes.phenotypes, dtype=np.float64)
    # jobs sharing a training set and λ are solved together (multi-RHS over traits)
    groups = {}
    for jb in jobs:
        key = (jb.idx_train.tobytes(), jb.lam if isinstance(jb.lam, str) else float(jb.lam))
        groups.setdefault(key, []).append(jb)
    for (_, lam), grp in groups.items():
        idx = grp[0].idx_train
        try:
            if idx.size < 2:
                raise ArgumentError("There are less than 2 entries with non-missing phenotype data after merging "
                                    "with the genotype data.")
            if lam == "reml":
                outs = []
                for jb in grp:
                    y = Yall[idx, jb.trait]
                    lj = session.reml(idx, y)["lambda"]
                    outs.append(session.gblup(idx, y, lj))
                fits = [(o[0][:, 0], o[1][:, 0]) for o in outs]
            else:
                Y = Yall[np.ix_(idx, [jb.trait for jb in grp])]
                b_hat, y_pred, mu, q = session.gblup(idx, Y, lam)
                fits = [(b_hat[:, k], y_pred[:, k]) for k in range(len(grp))]
            for jb, (b, yp) in zip(grp, fits):
                cv0 = cvs[jb.i]
                rows = jb.idx_train[jb.order]  # the caller's order, missing phenotypes dropped
                # a fresh Fit, as the model call of cvmultithread! returns (src/cross_validation.jl:170-177)
                f = Fit(n=rows.size, l=len(cv0.fit.b_hat_labels), model=cv0.fit.model,
                        b_hat_labels=list(cv0.fit.b_hat_labels), trait=cv0.fit.trait)
                f.entries = [genomes.entries[r] for r in rows]
                f.populations = [genomes.populations[r] for r in rows]
                f.b_hat = b.copy()
                f.y_pred = yp[jb.order].copy()
                f.y_true = Yall[rows, jb.trait].copy()
                f.metrics = metrics(f.y_true, f.y_pred)
                if not f.checkdims():
                    raise GBMError("Error fitting gblup.")
                yv_true = Yall[jb.idx_val, jb.trait]
                keep = np.isfinite(yv_true)
                iv = jb.idx_val[keep]
                yv_pred = _sorted_predict(session, iv, f.b_hat)
                cv = CV(cv0.replication, cv0.fold, f, [phenomes.populations[r] for r in iv],
                        [phenomes.entries[r] for r in iv], yv_true[keep], yv_pred, metrics(yv_true[keep], yv_pred))
                with lock:
                    cvs[jb.i] = cv
        except (GBMError, ArgumentError) as e:  # the reference warns and continues (src/cross_validation.jl:187-197)
            with lock:
                errors.append((grp[0].i, str(e)))


def cvmultithread(cvs, *, genomes: Genomes, phenomes: Phenomes, models_vector, verbose: bool = False,
                  devices=None):
    """Mirror of ``cvmultithread!`` (src/cross_validation.jl:151-207). GBLUP jobs run on one
    genotype session per device (one host thread each), grouped by training set so that the
    GRM is built once per set and traits sharing a set are solved together; other model
    callables run as in the reference (called with the six keywords, then ``validate``)."""
    if devices is None:
        devices = list(range(max(1, _lib.device_count())))
    pos_loci = {lab: k for k, lab in enumerate(genomes.loci_alleles)}
    pos_entry = {e: k for k, e in enumerate(genomes.entries)}
    gpu_jobs, other = [], []
    Yall = np.asarray(phenomes.phenotypes, dtype=np.float64)
    for i, (cv, model) in enumerate(zip(cvs, models_vector)):
        lam = _gblup_lambda(model)
        loci = [pos_loci[lab] for lab in cv.fit.b_hat_labels[1:]]
        if lam is not None and loci == list(range(len(genomes.loci_alleles))):
            gpu_jobs.append(_make_job(i, lam, [pos_entry[e] for e in cv.fit.entries],
                                      [pos_entry[e] for e in cv.validation_entries],
                                      phenomes.traits.index(cv.fit.trait), Yall))
        else:
            other.append((i, model, loci))
    errors, lock = [], threading.Lock()
    if gpu_jobs:
        # training sets go round-robin to devices, so the jobs that share one stay on one session
        keys = []
        for jb in gpu_jobs:
            k = jb.idx_train.tobytes()
            if k not in keys:
                keys.append(k)
        per_dev = {d: [] for d in range(len(devices))}
        for jb in gpu_jobs:
            per_dev[keys.index(jb.idx_train.tobytes()) % len(devices)].append(jb)
        X = np.asarray(genomes.allele_frequencies, dtype=np.float64)
        threads, sessions = [], []
        try:
            for d, jobs in per_dev.items():
                if not jobs:
                    continue
                s = GenotypeSession(X, device=devices[d])
                sessions.append(s)
                th = threading.Thread(target=_run_device_jobs, args=(s, jobs, cvs, genomes, phenomes, errors, lock))
                threads.append(th)
                th.start()
        finally:
            for th in threads:
                th.join()
            for s in sessions:
                s.close()
    for i, model, loci in other:
        cv = cvs[i]
        try:
            fit = model(genomes=genomes, phenomes=phenomes,
                        idx_entries=[genomes.entries.index(e) + 1 for e in cv.fit.entries],
                        idx_loci_alleles=[k + 1 for k in loci], idx_trait=phenomes.traits.index(cv.fit.trait) + 1,
                        verbose=False)
            cvs[i] = validate(fit, genomes, phenomes,
                              idx_validation=[genomes.entries.index(e) + 1 for e in cv.validation_entries],
                              replication=cv.replication, fold=cv.fold)
        except (GBMError, ArgumentError) as e:
            errors.append((i, str(e)))
    if verbose:
        for i, msg in errors:
            print(f"Warning: model fitting error in cross-validation job {i + 1}: {msg}")
    return cvs


def fold_assignments(n: int, n_folds: int, n_replications: int, n_traits: int, seed: int) -> np.ndarray:
    """idx_permutation per (trait, replication): folds 1..n_folds sampled with replacement
    (src/cross_validation.jl:359), shape (n_traits, n_replications, n)."""
    rng = np.random.default_rng(seed)
    out = np.empty((n_traits, n_replications, n), dtype=np.int64)
    for t in range(n_traits):
        for r in range(n_replications):
            out[t, r] = rng.integers(1, n_folds + 1, size=n)
    return out


def cvbulk_setup(*, genomes: Genomes, phenomes: Phenomes, models=(gblup,), n_replications: int = 5,
                 n_folds: int = 5, seed: int = 42):
    """Job setup of ``cvbulk`` (src/cross_validation.jl:282-398): argument checks, fold
    permutations, missing/zero-variance notes, one placeholder CV per (trait, replication, fold,
    model). Returns (cvs, notes, models_vector)."""
    if not genomes.checkdims() and not phenomes.checkdims():
        raise ArgumentError("The Genomes and Phenomes structs are corrupted ☹.")
    if not genomes.checkdims():
        raise ArgumentError("The Genomes struct is corrupted ☹.")
    if not phenomes.checkdims():
        raise ArgumentError("The Phenomes struct is corrupted ☹.")
    if list(genomes.entries) != list(phenomes.entries):
        raise ArgumentError("The genomes and phenomes input need to have been merged to have consitent entries.")
    if len(models) < 1:
        raise ArgumentError("No models were specified.")
    n, p = np.asarray(genomes.allele_frequencies).shape
    if n_folds < 1 or n_folds > n:
        raise ArgumentError(f"The number of folds, `n_folds = {n_folds}` is out of bounds. Please use values from 1 to {n}.")
    if n_replications < 1 or n_replications > 100:
        raise ArgumentError(f"The number of replications, `n_replications = {n_replications}` is out of bounds. "
                            "Please use values from 1 to 100.")
    perms = fold_assignments(n, n_folds, n_replications, len(phenomes.traits), seed)
    Y = np.asarray(phenomes.phenotypes, dtype=np.float64)
    cvs, notes, models_vector = [], [], []
    for t, trait in enumerate(phenomes.traits):
        phi = Y[:, t]
        ok = np.isfinite(phi)
        for r in range(n_replications):
            perm = perms[t, r]
            for j in range(1, n_folds + 1):
                idx_training = np.flatnonzero((perm != j) & ok)
                idx_validation = np.flatnonzero((perm == j) & ok)
                tag = [trait, f"replication_{r + 1}", f"fold_{j}"]
                if idx_training.size < 2 or idx_validation.size < 1:
                    notes.append(";".join(["too_many_missing"] + tag))
                    continue
                if phi[idx_training].var(ddof=1) < 1e-20:
                    notes.append(";".join(["zero_variance"] + tag))
                    continue
                for model in models:
                    fit = Fit(n=idx_training.size, l=p + 1)
                    fit.model = _model_label(model)
                    fit.trait = trait
                    fit.entries = [genomes.entries[i] for i in idx_training]
                    fit.populations = [genomes.populations[i] for i in idx_training]
                    fit.b_hat_labels = ["intercept"] + list(genomes.loci_alleles)
                    m = idx_validation.size
                    cvs.append(CV(f"replication_{r + 1}", f"fold_{j}", fit,
                                  [genomes.populations[i] for i in idx_validation],
                                  [genomes.entries[i] for i in idx_validation], np.zeros(m), np.zeros(m),
                                  dict(fit.metrics)))
                    models_vector.append(model)
    return cvs, notes, models_vector


def cvbulk(*, genomes: Genomes, phenomes: Phenomes, models=(gblup,), n_replications: int = 5, n_folds: int = 5,
           seed: int = 42, verbose: bool = False, devices=None):
    """Mirror of ``cvbulk`` (src/cross_validation.jl:268-401): replicated k-fold CV across all
    traits and entries. Returns (cvs, notes)."""
    cvs, notes, models_vector = cvbulk_setup(genomes=genomes, phenomes=phenomes, models=models,
                                             n_replications=n_replications, n_folds=n_folds, seed=seed)
    if verbose:
        print("Setup", len(cvs), "cross-validation job/s.")
        print("Skipping", len(notes), "cross-validation job/s.")
    cvmultithread(cvs, genomes=genomes, phenomes=phenomes, models_vector=models_vector, verbose=verbose,
                  devices=devices)
    return cvs, notes
