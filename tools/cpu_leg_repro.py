#!/usr/bin/env python3
"""Re-run bench.py's CPU legs (and the OpenBLAS calls they make at C3's n = 50 000) on the host cores of a GPU
box, each in a spawned child with faulthandler on, and report the exit code / signal of every child: the hunt for
the one bench run that died with SIGSEGV in round 4. Touches no GPU.

    python tools/cpu_leg_repro.py [--reps 3] > gpurun_out/cpu_leg_repro.jsonl
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _numpy_syrk(n, p):
    import numpy as np
    Z = np.random.default_rng(0).standard_normal((n, p))
    G = Z @ Z.T  # numpy's A @ A.T → ILP64 OpenBLAS dsyrk
    return float(G[-1, -1] - (Z[-1] ** 2).sum())


def _scipy_syrk(n, p):
    import numpy as np
    import scipy.linalg as sla
    Z = np.asfortranarray(np.random.default_rng(0).standard_normal((n, p)))
    G = sla.blas.dsyrk(1.0, Z)  # scipy's LP64 OpenBLAS
    return float(G[-1, -1] - (Z[-1] ** 2).sum())


def _c2_leg(_):
    sys.path.insert(0, ROOT)
    import numpy as np
    import bench

    class A:
        individuals, loci, cpu_sample_p, seed, nrhs, lam = 5000, 50000, 0, 4242, 1, 1.0
    Y = np.random.default_rng(0).standard_normal((5000, 1))
    gpu = {"y_pred": np.zeros((5000, 1)), "mu": np.zeros(1), "q": 50000, "b_hat": np.zeros((50001, 1))}
    out, _, _ = bench.cpu_baseline(A(), Y, gpu)
    return out["value"]


def _child(name, arg, q):
    import faulthandler
    faulthandler.enable()
    fn = {"numpy_syrk": lambda a: _numpy_syrk(*a), "scipy_syrk": lambda a: _scipy_syrk(*a), "c2_leg": _c2_leg}[name]
    t0 = time.time()
    q.put({"result": fn(arg), "seconds": time.time() - t0})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from threadpoolctl import threadpool_info
    import numpy  # noqa: F401
    import scipy.linalg  # noqa: F401
    cpu = next((ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")), "?")
    print(json.dumps({"cpu": cpu, "nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
                      "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"),
                      "blas": [{k: d.get(k) for k in ("filepath", "version", "architecture", "num_threads")}
                               for d in threadpool_info()]}), flush=True)
    ctx = mp.get_context("spawn")
    jobs = [("numpy_syrk", (50000, 64)), ("scipy_syrk", (50000, 64)), ("numpy_syrk", (46341, 256)), ("c2_leg", None)]
    for rep in range(args.reps):
        for name, arg in jobs:
            q = ctx.Queue()
            p = ctx.Process(target=_child, args=(name, arg, q))
            p.start()
            p.join(900)
            res = q.get() if not q.empty() else None
            print(json.dumps({"rep": rep, "leg": name, "arg": arg, "exit_code": p.exitcode, "out": res}), flush=True)


if __name__ == "__main__":
    main()
