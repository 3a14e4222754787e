"""Per-unit timeline of the persistent GRM kernel (debug build -DGBM_DEBUG_WGTIME through
GBM_LIBGBM): µs per 16-locus stage by loci range, slot busy fraction, gaps between units."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
import torch  # noqa: E402

from gbm.sharded import HipShardStages  # noqa: E402

n, p = (int(a) for a in sys.argv[1:3]) if len(sys.argv) > 2 else (5000, 50000)
st = HipShardStages(n, p)
st.generate(4242, 0)
st.standardize()
for _ in range(3):
    st.grm_syrk()
torch.cuda.synchronize()
buf = np.zeros(3 * 16384, dtype=np.uint64)
st.lib.gbm_debug_wgtime.argtypes = [ctypes.c_void_p, ctypes.c_int64]
assert st.lib.gbm_debug_wgtime(buf.ctypes.data, 16384) == 0
t = buf.reshape(-1, 3).astype(np.int64)
idx = np.nonzero(t[:, 1] > 0)[0]
s, e, hw = t[idx, 0], t[idx, 1], t[idx, 2]
base = s.min()
s, e = (s - base) / 100.0, (e - base) / 100.0
xcc, cu, wg = hw & 0xFF, (hw >> 8) & 0xFF, (hw >> 16) & 0xFFF
cyc = hw >> 28  # s_memtime ticks over the unit
nt = (n + 127) // 128
if nt >= 8 and n - (nt - 1) * 128 <= 64:
    nt -= 1
ntiles = nt * (nt + 1) // 2
sl = idx // ntiles
T = e.max()
print(f"n={n} p={p} units={len(idx)} makespan {T/1e3:.3f} ms, workgroups {len(np.unique(wg))}")
# stage counts per range from the plan (GBM_DEBUG_PLAN is not needed: infer from durations' order)
for r in range(sl.max() + 1):
    m = sl == r
    d = e[m] - s[m]
    f = cyc[m] / (d * 1e-6) / 1e9  # GHz of the s_memtime counter
    print(f"range {r}: units {m.sum()} start {np.percentile(s[m], [0, 50, 100]).round(0)} dur med {np.median(d):.1f} "
          f"p5 {np.percentile(d, 5):.1f} p95 {np.percentile(d, 95):.1f} us; memtime rate med {np.median(f):.3f} "
          f"p5 {np.percentile(f, 5):.3f} p95 {np.percentile(f, 95):.3f} GHz")
busy = np.zeros(wg.max() + 1)
gaps = []
for w in np.unique(wg):
    m = wg == w
    o = np.argsort(s[m])
    ss, ee = s[m][o], e[m][o]
    busy[w] = (ee - ss).sum()
    gaps.extend(list(ss[1:] - ee[:-1]))
    busy[w] = busy[w]
print(f"slot busy fraction {busy.sum() / (len(np.unique(wg)) * T):.3f}; gap between units med {np.median(gaps):.2f} "
      f"p95 {np.percentile(gaps, 95):.2f} us; last unit end per xcc:",
      [round(e[xcc == x].max() / 1e3, 3) for x in range(8)])

# which units are slow: per-stage time vs xcc, CU, tile column, diag, start time
tt = idx % ntiles
tj = np.floor((np.sqrt(8.0 * tt + 1.0) - 1.0) / 2.0).astype(np.int64)
tj = np.where((tj + 1) * (tj + 2) // 2 <= tt, tj + 1, tj)
tj = np.where(tj * (tj + 1) // 2 > tt, tj - 1, tj)
ti = tt - tj * (tj + 1) // 2
d = e - s
for r in range(sl.max() + 1):
    m = sl == r
    ref = np.median(d[m])
    slow = m & (d > 1.08 * np.percentile(d[m], 10))
    print(f"range {r}: slow units {slow.sum()}/{m.sum()}; slow frac by xcc", [round(float(slow[xcc == x].sum()) / max(1, (m & (xcc == x)).sum()), 2) for x in range(8)])
# per CU (xcc, cu): fraction of slow units across all ranges, and whether the two slots of a CU differ
key = xcc * 256 + cu
slowall = np.zeros(len(d), bool)
for r in range(sl.max() + 1):
    m = sl == r
    slowall |= m & (d > 1.08 * np.percentile(d[m], 10))
ks = np.unique(key)
fr = np.array([slowall[key == k].mean() for k in ks])
print("per-CU slow fraction quantiles", np.percentile(fr, [0, 10, 50, 90, 100]).round(2), "CUs", len(ks))
wgs = np.unique(wg)
fw = np.array([slowall[wg == w].mean() for w in wgs])
print("per-WG slow fraction quantiles", np.percentile(fw, [0, 10, 50, 90, 100]).round(2))
print("slow frac diag", slowall[ti == tj].mean().round(2), "offdiag", slowall[ti != tj].mean().round(2))
