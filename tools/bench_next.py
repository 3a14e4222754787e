"""Timings of the §8f rows on one GPU (not the driver's bench): cross-validation fold farming
(C5-shaped), REML λ, ridge path (C1) and the BRR Gibbs sampler (C4-shaped). Prints one JSON
line per measurement. Sizes via flags; defaults finish in a few minutes."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def synth(n, p, seed, t=1):
    import oracle
    X = oracle.synth_genotypes(seed, n, p)
    return X, oracle.synth_phenotypes(X, seed + 1, ntraits=t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["cv", "reml", "ridge", "brr"])
    ap.add_argument("--n", type=int, default=5000)
    ap.add_argument("--p", type=int, default=50000)
    ap.add_argument("--traits", type=int, default=3)
    ap.add_argument("--folds", type=int, default=10)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime)
    import gbm
    X, Y = synth(args.n, args.p, 4242, args.traits)
    if args.what == "cv":
        ent = [f"e{i}" for i in range(args.n)]
        g = gbm.Genomes(ent, ["p"] * args.n, [f"l{j}" for j in range(args.p)], X)
        ph = gbm.Phenomes(ent, ["p"] * args.n, [f"t{k}" for k in range(args.traits)], Y)
        t0 = time.perf_counter()
        cvs, notes = gbm.cvbulk(genomes=g, phenomes=ph, n_replications=1, n_folds=args.folds, seed=42)
        dt = time.perf_counter() - t0
        print(json.dumps({"bench": "cvbulk gblup", "n": args.n, "p": args.p, "traits": args.traits,
                          "folds": args.folds, "jobs": len(cvs), "seconds": dt, "s_per_fold_job": dt / len(cvs),
                          "mean_cor": float(np.mean([c.metrics["cor"] for c in cvs]))}))
    elif args.what == "reml":
        with gbm.GenotypeSession(X) as s:
            idx = np.arange(args.n)
            s.gblup(idx, Y[:, 0], 1.0)  # GRM build (cached)
            t0 = time.perf_counter()
            r = s.reml(idx, Y[:, 0])
            dt = time.perf_counter() - t0
        print(json.dumps({"bench": "reml lambda (GRM cached)", "n": args.n, "p": args.p, "seconds": dt, **r}))
    elif args.what == "ridge":
        t0 = time.perf_counter()
        out = gbm.ridge_path_cv(X, Y[:, 0])
        dt = time.perf_counter() - t0
        print(json.dumps({"bench": "ridge glmnetcv path (100 lambda x (1 + folds))", "n": args.n, "p": args.p,
                          "seconds": dt, "argmin": int(np.argmin(out["meanloss"]))}))
    else:
        t0 = time.perf_counter()
        b, yp, var = gbm.brr_arrays(X, Y[:, 0], n_iter=args.iters, n_burnin=args.iters // 2, thin=1)
        dt = time.perf_counter() - t0
        print(json.dumps({"bench": "BRR Gibbs", "n": args.n, "p": args.p, "iters": args.iters, "seconds": dt,
                          "ms_per_iter_incl_setup": dt / args.iters * 1e3,
                          "cor": float(np.corrcoef(yp, Y[:, 0])[0, 1])}))


if __name__ == "__main__":
    main()
