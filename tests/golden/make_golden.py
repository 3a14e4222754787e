"""Generate the committed golden fixtures from the CPU oracle (oracle/oracle.py, numpy/LAPACK fp64).

Parity status: these vectors pin the oracle and the HIP path against each other and against
regressions; they are NOT reference (Julia) outputs — the reference cannot run here and ships no
numeric fixtures, so parity with GenomicBreedingModels.jl itself is
"unpinned". Re-run with: python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle  # noqa: E402


def dosage_case(name, seed, n, p, ntraits, lam, monomorphic=(), missing=0):
    X = oracle.synth_genotypes(seed, n, p)  # dosage/2 exactly
    for j, v in monomorphic:
        X[:, j] = v
    D = np.round(X * 2).astype(np.int8)
    assert np.array_equal(D / 2.0, X)
    Y = oracle.synth_phenotypes(X, seed + 1, ntraits=ntraits)
    Yfull = Y.copy()
    keep_rows = np.ones(n, dtype=bool)
    if missing:
        rng = np.random.default_rng(seed + 2)
        miss = rng.choice(n, size=missing, replace=False)
        Yfull[miss, 0] = np.nan
        keep_rows[miss] = False
    Xk, Yk = X[keep_rows], Yfull[keep_rows]
    r = oracle.gblup_fit(Xk, Yk, lam)
    G = r["G"]
    met = [oracle.metrics(Yk[:, t], r["y_pred"][:, t]) for t in range(ntraits)]
    np.savez_compressed(
        os.path.join(HERE, f"{name}.npz"),
        dosage=D, ploidy=np.int64(2), phenotypes=Yfull, lam=np.float64(lam), keep_rows=keep_rows,
        q=np.int64(r["q"]), mu=r["mu"], y_pred=r["y_pred"], b_hat=r["b_hat"], a=r["a"],
        mean=r["mean"], sd=r["sd"], keep=r["keep"],
        G_trace=np.float64(np.trace(G)), G_sum=np.float64(G.sum()), G_first_row=G[0].copy(),
        G_diag=np.diag(G).copy(),
        metrics_json=np.array(json.dumps(met)),
    )
    print(name, X.shape, "q =", r["q"], "mu =", r["mu"])


if __name__ == "__main__":
    dosage_case("c1_200x1000", 42, 200, 1000, 1, 1.0)
    dosage_case("ragged_333x1777_3traits", 7, 333, 1777, 3, 0.5,
                monomorphic=[(0, 0.0), (100, 0.5), (1776, 1.0)])
    dosage_case("missing_150x600", 9, 150, 600, 1, 2.0, missing=17)
