"""Two SNP-column shards through the C-ABI host entry (gbm_gblup_fit, devices=[0, 0], X in pageable
host memory, the Julia ccall path with devices=[0..7] rehearsed on one GPU): the shards driven one
after the other (GBM_SHARD_THREADS=0, round 2's schedule) against one host thread per shard (round
3). Prints one JSON line; run it under rocprofv3 --kernel-trace --memory-copy-trace to see shard 1's
host-to-device copies overlap shard 0's GRM (tools/overlap_from_trace.py reads the trace).
Timing tool only."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
import numpy as np  # noqa: E402

import gbm  # noqa: E402
from gbm import _lib, synth  # noqa: E402

n, p, seed = int(os.environ.get("N", "5000")), int(os.environ.get("P", "50000")), 4242
reps = int(os.environ.get("REPS", "3"))
modes = os.environ.get("MODES", "0,1").split(",")
Y = np.asfortranarray(synth.qtl_phenotypes(seed, n, p, 1))
X = synth.genotypes(seed, n, p)
lib = gbm.load_library()
b = np.zeros((p + 1, 1), order="F")
yp = np.zeros((n, 1), order="F")
mu = np.zeros(1)
q = np.zeros(1, dtype=np.int64)
devs, nd = _lib.devices_arg([0, 0])
out = {"tool": "two_shard_overlap", "n": n, "p": p, "devices": [0, 0], "x_gb": X.nbytes / 1e9}


def fit():
    _lib.check(lib.gbm_gblup_fit(_lib.ptr(X), n, p, n, _lib.ptr(Y), n, 1, 1.0, devs, nd, _lib.ptr(b), _lib.ptr(yp),
                                 _lib.ptr(mu), _lib.ptr(q)), "gbm_gblup_fit")


res = {}
for mode in modes:
    os.environ["GBM_SHARD_THREADS"] = mode
    fit()  # warm-up (pooled contexts)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fit()
        ts.append(time.perf_counter() - t0)
    res[mode] = yp.copy()
    out["ms_serial" if mode == "0" else "ms_threaded"] = 1e3 * float(np.median(ts))
if len(res) == 2:
    out["bit_identical"] = bool(np.array_equal(res["0"], res["1"]))
print(json.dumps(out), flush=True)
