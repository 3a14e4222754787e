"""Synthetic benchmark data from libgbm's device generator: counter-hash genotypes
(MAF f ~ U(0.05, 0.5), dosage ~ Binomial(2, f), X = dosage/2) and 1 %-QTL phenotypes (h² = 0.5).
The generator is a pure function of (seed, individual, locus), so any rank or process can
materialise any block of loci without communication. Benchmark plumbing, not a model path."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib


def _torch():
    import torch
    return torch


def genotypes_device(seed: int, n: int, p: int, j0: int = 0, device: int = 0):
    """Loci j0 .. j0+p-1 as a (p, npad(n)) float64 torch tensor on `device` (locus rows, padding zero)."""
    torch = _torch()
    lib = _lib.load()
    dev = torch.device("cuda", device)
    npad = lib.gbm_dev_npad(n)
    Xt = torch.empty((p, npad), dtype=torch.float64, device=dev)
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(lib.gbm_dev_synth_genotypes(ctypes.c_void_p(Xt.data_ptr()), npad, p, n, int(seed), int(j0), stream),
               "gbm_dev_synth_genotypes")
    return Xt


def genotypes(seed: int, n: int, p: int, j0: int = 0, device: int = 0) -> np.ndarray:
    """X (n x p, column-major like Julia) of loci j0 .. j0+p-1, generated on the device."""
    Xt = genotypes_device(seed, n, p, j0, device)
    return np.asfortranarray(Xt[:, :n].cpu().numpy().T)


def qtl_phenotypes(seed: int, n: int, p_total: int, ntraits: int = 1, device: int = 0) -> np.ndarray:
    """Y (n x ntraits): y = Xβ + e over 1 % QTL loci of [0, p_total) with β ~ N(0, 1) and
    e ~ N(0, var(g)) (h² = 0.5); the QTL columns come from the device generator, so every rank
    builds the same Y without communication."""
    torch = _torch()
    lib = _lib.load()
    dev = torch.device("cuda", device)
    npad = lib.gbm_dev_npad(n)
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    rng = np.random.default_rng(seed + 1)
    Y = np.empty((n, ntraits))
    for t in range(ntraits):
        nq = max(1, p_total // 100)
        idx = np.sort(rng.choice(p_total, size=nq, replace=False))
        beta = rng.standard_normal(nq)
        Xq = torch.empty((nq, npad), dtype=torch.float64, device=dev)
        for k, j in enumerate(idx):
            _lib.check(lib.gbm_dev_synth_genotypes(ctypes.c_void_p(Xq[k].data_ptr()), npad, 1, n, int(seed), int(j),
                                                   stream), "gbm_dev_synth_genotypes")
        Xq = Xq[:, :n].cpu().numpy()
        g = np.zeros(n)
        for k in range(nq):  # fixed summation order: identical on every rank
            g += Xq[k] * beta[k]
        e = rng.standard_normal(n) * np.sqrt(g.var(ddof=1))
        Y[:, t] = g + e
    return Y
