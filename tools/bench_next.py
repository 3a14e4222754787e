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


def synth(n, p, seed, t=1):
    """Host X and Y from libgbm's device generator (gbm.synth)."""
    from gbm import synth as S
    return S.genotypes(seed, n, p), S.qtl_phenotypes(seed, n, p, ntraits=t)


def cv_sessions(args):
    """C5-shaped fold farming at full size: synthetic genotypes generated on each device (no host
    X), one session per device, the (trait, fold) jobs grouped by training set and dealt
    round-robin to the devices, one host thread per device (the cvbulk scheme, src/cross_validation.jl:345-401)."""
    import threading

    import gbm
    from gbm import synth as S
    ndev = args.devices
    Y = S.qtl_phenotypes(4242, args.n, args.p, ntraits=args.traits)
    folds = gbm.fold_assignments(args.n, args.folds, 1, args.traits, 42)[:, 0]  # (traits, n)
    jobs = [(t, f) for t in range(args.traits) for f in range(1, args.folds + 1)]
    t0 = time.perf_counter()
    sessions = [gbm.GenotypeSession.synthetic(4242, args.n, args.p, device=d) for d in range(ndev)]
    t_setup = time.perf_counter() - t0
    cors = {}
    errs = []

    def worker(d):
        try:
            for k, (t, f) in enumerate(jobs):
                if k % ndev != d:
                    continue
                tr = np.nonzero(folds[t] != f)[0]
                va = np.nonzero(folds[t] == f)[0]
                b_hat, _, _, _ = sessions[d].gblup(tr, Y[tr, t], 1.0)
                yp = sessions[d].predict(va, b_hat[:, 0])
                cors[(t, f)] = float(np.corrcoef(yp, Y[va, t])[0, 1])
        except Exception as e:  # pragma: no cover - reported below
            errs.append(repr(e))

    t1 = time.perf_counter()
    th = [threading.Thread(target=worker, args=(d,)) for d in range(ndev)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t1
    for s in sessions:
        s.close()
    if errs:
        raise RuntimeError(errs[0])
    import os
    print(json.dumps({"bench": "cv fold farming on synthetic sessions", "grm": os.environ.get("GBM_GRM", "fp64"),
                      "n": args.n, "p": args.p,
                      "traits": args.traits, "folds": args.folds, "devices": ndev, "jobs": len(jobs),
                      "session_setup_s": t_setup, "seconds": dt, "s_per_fold_job": dt / len(jobs) * ndev,
                      "mean_cor": float(np.mean(list(cors.values())))}), flush=True)


def brr_sessionless(args):
    """C4-shaped BRR: n x p synthetic genotypes, a few Gibbs iterations timed (the per-iteration
    cost is constant, so 5 000 iterations = 5 000 x this)."""
    import gbm
    X, Y = synth(args.n, args.p, 4242, 1)
    res = {}
    for iters in (args.iters // 5, args.iters):
        t0 = time.perf_counter()
        b, yp, var = gbm.brr_arrays(X, Y[:, 0], n_iter=iters, n_burnin=iters // 2, thin=1)
        res[iters] = time.perf_counter() - t0
    lo, hi = args.iters // 5, args.iters
    per = (res[hi] - res[lo]) / (hi - lo)
    print(json.dumps({"bench": "BRR Gibbs (C4 shape)", "n": args.n, "p": args.p, "iters": [lo, hi],
                      "seconds": [res[lo], res[hi]], "ms_per_iter": per * 1e3,
                      "projected_5000_iter_s": res[lo] + per * (5000 - lo),
                      "cor": float(np.corrcoef(yp, Y[:, 0])[0, 1])}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["cv", "reml", "ridge", "brr", "cv-synth", "brr-c4"])
    ap.add_argument("--n", type=int, default=5000)
    ap.add_argument("--p", type=int, default=50000)
    ap.add_argument("--traits", type=int, default=3)
    ap.add_argument("--folds", type=int, default=10)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--devices", type=int, default=1)
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime)
    import gbm
    if args.what == "cv-synth":
        return cv_sessions(args)
    if args.what == "brr-c4":
        return brr_sessionless(args)
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
