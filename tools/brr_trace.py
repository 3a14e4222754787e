"""Phase timeline of the BRR super-block sweep (GBM_BRR_TRACE=1): runs a C4-shape fit for a few
iterations and prints, for workgroups 0 and C − 1 of the last sweep, the mean time per super-block
of each phase (dots + publish, hand-off 1 wait, r̃ + publish, hand-off 2 wait, δ + b + publish,
hand-off 3 wait, e update). Timing tool only; one JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
os.environ["GBM_BRR_TRACE"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import gbm  # noqa: E402
from gbm import synth  # noqa: E402

n, p = int(os.environ.get("N", "10000")), int(os.environ.get("P", "100000"))
X = synth.genotypes(4242, n, p)
y = synth.qtl_phenotypes(4242, n, p, 1)[:, 0]
gbm.brr_arrays(X, y, n_iter=6, n_burnin=2, thin=1)
lib = gbm.load_library()
nsb = (p + 511) // 512
buf = np.zeros(2 * nsb * 12, dtype=np.int64)
lib.gbm_debug_brr_trace.restype = ctypes.c_int64
got = lib.gbm_debug_brr_trace(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(buf.size))
names = ["dots+publish", "wait1", "rtilde+publish", "wait2", "delta+publish", "wait3", "e_update"]
sub = {"e_slices": (6, 8), "e_dma_wait+barrier": (8, 9), "e_reduce": (9, 10), "e_apply": (10, 7)}
out = {"tool": "brr_trace", "n": n, "p": p, "nsb": nsb, "records": int(got)}
for w, tag in ((0, "wg0"), (1, "wg_last")):
    t = buf[w * nsb * 12:(w + 1) * nsb * 12].reshape(nsb, 12).astype(np.float64) * 10.0  # 100 MHz ticks -> ns
    d = np.diff(t[:, :8], axis=1)
    out[tag] = {k: float(np.mean(d[1:, i]) / 1000.0) for i, k in enumerate(names)}  # µs
    for k, (a, b) in sub.items():
        out[tag][k] = float(np.mean(t[1:, b] - t[1:, a]) / 1000.0)
    out[tag]["sb_total_us"] = float(np.mean(t[2:, 0] - t[1:-1, 0]) / 1000.0)
print(json.dumps(out))
