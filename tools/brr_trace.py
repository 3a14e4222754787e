"""Phase timeline of the BRR super-block sweep (GBM_BRR_TRACE=1, path 4): runs a C4-shape fit for a
few iterations and prints per-workgroup mean times per super-block of the steps (A) δ + partial
gathers, (B) C δ + r̃ publish, (C) e update + dots (of super-block s + 2), (D) r̃ gather + δ publish.
Timing tool only; one JSON line."""
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
path, fb = ctypes.c_int(-1), ctypes.c_int64(0)
lib.gbm_debug_brr_stats(ctypes.byref(path), ctypes.byref(fb))
sh = [ctypes.c_int(0) for _ in range(5)]
lib.gbm_debug_brr_shape(*[ctypes.byref(v) for v in sh])
C, O, R, Ko, Kn = [v.value for v in sh]
cap = max(2 * nsb * 12, C * nsb * 8)
buf = np.zeros(cap, dtype=np.int64)
lib.gbm_debug_brr_trace.restype = ctypes.c_int64
got = lib.gbm_debug_brr_trace(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(buf.size))
out = {"tool": "brr_trace", "n": n, "p": p, "nsb": nsb, "records": int(got), "path": path.value,
       "shape": {"C": C, "O": O, "R": R, "Ko": Ko, "Kn": Kn}}
if path.value in (3, 4):
    # every workgroup: marks 0 A end (δ_{s−1} seen), 1 B end (r̃ published), 5 e update end, 2 C end (P_{s+1}
    # published), 4 δ_s published, 3 step end (Q_{s+1} gathered); 100 MHz ticks -> µs
    T = buf[:C * nsb * 8].reshape(C, nsb, 8).astype(np.float64) / 100.0
    own = np.arange(C) < O
    for w, tag in ((0, "wg0"), (C - 1, "wg_last")):
        t = T[w]
        prev = np.concatenate([[t[0, 0]], t[:-1, 3]])
        ph = {"A_delta_gather": t[:, 0] - prev, "B_cdelta_rtilde": t[:, 1] - t[:, 0], "C_eupdate": t[:, 5] - t[:, 1],
              "C_dots": t[:, 2] - t[:, 5], "D_rtilde_gather_delta": t[:, 4] - t[:, 2], "D_q_gather": t[:, 3] - t[:, 4]}
        if path.value == 4:  # e update sub-phases: 6 slices done, 7 reduction done
            ph.update({"C_e_slices": t[:, 6] - t[:, 1], "C_e_reduce": t[:, 7] - t[:, 6], "C_e_apply": t[:, 5] - t[:, 7]})
        if not own[w]:
            ph = {k: v for k, v in ph.items() if not k.startswith("D")}
            ph["C_to_step_end"] = t[:, 3] - t[:, 2]
        out[tag] = {k: float(np.mean(v[2:-2])) for k, v in ph.items()}
        out[tag]["sb_total_us"] = float(np.mean(np.diff(t[:, 3])[2:-2]))
    s = slice(2, nsb - 2)
    a_end = T[:, s, 0]          # δ_{s−1} seen
    p_pub = T[:, s, 2]          # P_{s+1} published
    d_pub = T[own][:, s, 4]     # δ_s published (owners)
    q_end = T[own][:, s, 3]     # Q_{s+1} gathered (owners)
    out["skew"] = {
        "delta_seen_spread_us": float(np.mean(a_end.max(0) - a_end.min(0))),
        "P_publish_spread_us": float(np.mean(p_pub.max(0) - p_pub.min(0))),
        "P_last_publish_minus_first_delta_seen_us": float(np.mean(p_pub.max(0) - a_end.min(0))),
        "owners_q_end_minus_last_P_publish_us": float(np.mean(q_end.max(0) - p_pub.max(0))),
        "owners_delta_publish_spread_us": float(np.mean(d_pub.max(0) - d_pub.min(0))),
        "slowest_P_publisher_counts": np.bincount(np.argmax(p_pub, 0), minlength=C).argsort()[-5:][::-1].tolist(),
    }
    # hop δ: last owner's δ_s publish -> each workgroup's A end of step s + 1
    dp = T[own][:, :, 4].max(0)  # per s
    hop = T[:, 3:nsb - 1, 0] - dp[None, 2:nsb - 2]
    out["skew"]["delta_hop_us_mean_min_max"] = [float(hop.mean()), float(hop.min(1).mean()), float(hop.max(0).mean())]
else:
    for w, tag in ((0, "wg0"), (1, "wg_last")):
        t = buf[w * nsb * 12:(w + 1) * nsb * 12].reshape(nsb, 12).astype(np.float64) * 10.0  # 100 MHz ticks -> ns
        names = ["dots+publish", "wait1", "rtilde+publish", "wait2", "delta+publish", "wait3", "e_update"]
        sub = {"e_slices": (6, 8), "e_dma_wait+barrier": (8, 9), "e_reduce": (9, 10), "e_apply": (10, 7)}
        d = np.diff(t[:, :8], axis=1)
        out[tag] = {k: float(np.mean(d[1:, i]) / 1000.0) for i, k in enumerate(names)}  # µs
        for k, (a, b) in sub.items():
            out[tag][k] = float(np.mean(t[1:, b] - t[1:, a]) / 1000.0)
        out[tag]["sb_total_us"] = float(np.mean(t[2:, 0] - t[1:-1, 0]) / 1000.0)
print(json.dumps(out))
