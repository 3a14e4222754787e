"""Per-workgroup timeline of the GRM SYRK (debug build with -DGBM_DEBUG_WGTIME, loaded through
GBM_LIBGBM): steady-state per-stage time, occupancy of the resident slots, tail length, XCD spread."""
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
t = buf.reshape(-1, 3)
t = t[t[:, 1] > 0]
nwg = len(t)
t0, t1, hw = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64), t[:, 2]
base = t0.min()
s, e = (t0 - base) / 100.0, (t1 - base) / 100.0  # µs (100 MHz)
xcc = (hw >> 32) & 0xF
cu = (hw >> 8) & 0xF
se = (hw >> 13) & 0x7
dur = e - s
kernel = e.max()
print(f"n={n} p={p} persistent wgs={nwg} first-start..last-end {kernel/1e3:.3f} ms")
print("start quantiles (us):", np.percentile(s, [0, 50, 90, 99, 100]).round(1))
print("end quantiles (us):", np.percentile(e, [0, 5, 50, 95, 100]).round(1))
print("duration quantiles (us):", np.percentile(dur, [0, 5, 50, 95, 100]).round(1))
print(f"slot occupancy sum(dur)/(512*T) = {dur.sum() / (min(nwg, 512) * kernel):.3f}")
for x in range(8):
    m = xcc == x
    print(f"xcc {x}: wgs {m.sum()} end max {e[m].max():.1f} median dur {np.median(dur[m]):.1f} min {dur[m].min():.1f}")
# pairs sharing a CU
key = (xcc.astype(np.int64) << 8) | ((hw >> 8) & 0xFF).astype(np.int64)
u, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
print("WGs per (xcc, se/sh/cu) slot histogram:", np.bincount(cnt))
# per tile class within each loci slice: interior, diagonal, ragged last tile column (tj = nt-1)
nt = (n + 127) // 128
if nt >= 8 and n - (nt - 1) * 128 <= 64 and os.environ.get("GBM_GRM_EDGE", "1") != "0":
    nt -= 1  # ragged last column handled by grm_edge_kernel
ntiles = nt * (nt + 1) // 2
T8 = (ntiles + 7) & ~7
wg_all = np.arange(len(buf) // 3)
rec = buf.reshape(-1, 3)[:, 1] > 0
wgi = wg_all[rec]
sl = wgi // T8
u = wgi - sl * T8
tt = (u & 7) * (T8 >> 3) + (u >> 3)
tj = np.floor((np.sqrt(8.0 * tt + 1.0) - 1.0) / 2.0).astype(np.int64)
tj = np.where((tj + 1) * (tj + 2) // 2 <= tt, tj + 1, tj)
tj = np.where(tj * (tj + 1) // 2 > tt, tj - 1, tj)
ti = tt - tj * (tj + 1) // 2
for s_ in range(int(sl.max()) + 1):
    m = sl == s_
    inter = m & (ti != tj) & (tj != nt - 1)
    dg = m & (ti == tj) & (tj != nt - 1)
    edge = m & (tj == nt - 1)
    print(f"slice {s_}: interior n={inter.sum()} med {np.median(dur[inter]):.1f} us | diag {np.median(dur[dg]) if dg.any() else 0:.1f}"
          f" | last column n={edge.sum()} med {np.median(dur[edge]) if edge.any() else 0:.1f} us (ragged cols {n - (nt - 1) * 128})")
