"""C3 per-GPU shape through the C-ABI host entry (the Julia ccall path): gbm_gblup_fit with X in
pageable host memory (n = 50 000 x p = 75 000 loci = C3's share of one GPU, 30 GB fp64) and
gbm_gblup_fit_dosage_i8 with int8 dosages (3.75 GB). Timing tool only; prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gbm  # noqa: E402
from gbm import _lib, synth  # noqa: E402

n, p, seed = int(os.environ.get("N", "50000")), int(os.environ.get("P", "75000")), 424242
Y = np.asfortranarray(synth.qtl_phenotypes(seed, n, p, 1))
X = synth.genotypes(seed, n, p)  # (n, p) column-major, host
torch.cuda.empty_cache()
lib = gbm.load_library()
b = np.zeros((p + 1, 1), order="F")
yp = np.zeros((n, 1), order="F")
mu = np.zeros(1)
q = np.zeros(1, dtype=np.int64)
out = {"tool": "c3_host_path", "n": n, "p": p, "x_gb": X.nbytes / 1e9}


def timed(fn):
    t0 = time.perf_counter()
    fn()
    return time.perf_counter() - t0


f64 = lambda: _lib.check(lib.gbm_gblup_fit(_lib.ptr(X), n, p, n, _lib.ptr(Y), n, 1, 1.0, None, 0, _lib.ptr(b),
                                           _lib.ptr(yp), _lib.ptr(mu), _lib.ptr(q)), "gbm_gblup_fit")
out["f64_first_call_s"] = timed(f64)
out["f64_call_s"] = timed(f64)
y64 = yp.copy()
D = np.asfortranarray(np.rint(X * 2.0).astype(np.int8))
del X
i8 = lambda: _lib.check(lib.gbm_gblup_fit_dosage_i8(_lib.ptr(D), n, p, n, 2, _lib.ptr(Y), n, 1, 1.0, None, 0,
                                                    _lib.ptr(b), _lib.ptr(yp), _lib.ptr(mu), _lib.ptr(q)),
                        "gbm_gblup_fit_dosage_i8")
out["i8_call_s"] = timed(i8)
out["i8_vs_f64_max_rel"] = float(np.abs(yp - y64).max() / np.abs(y64).max())
out["q"] = int(q[0])
flops = float(n) * (n + 1) * p + n ** 3 / 3.0
out["f64_tflops_e2e"] = flops / out["f64_call_s"] / 1e12
out["i8_tflops_e2e"] = flops / out["i8_call_s"] / 1e12
print(json.dumps(out), flush=True)
