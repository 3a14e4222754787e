"""Phases of the diagonal-block factor inside the small trailing-update kernel (debug build with
-DGBM_DEBUG_FACTIME loaded through GBM_LIBGBM): one solve at n, then per launch
tile (kernel start -> factor start), factor_diag_block, store_factor, in µs."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
import torch  # noqa: E402,F401

from gbm.sharded import HipShardStages  # noqa: E402

n, p = (int(a) for a in sys.argv[1:3]) if len(sys.argv) > 2 else (5000, 20000)
st = HipShardStages(n, p)
st.generate(4242, 0)
st.load_phenotypes(np.random.default_rng(0).standard_normal((n, 1)))
st.standardize()
st.grm_syrk()
st.grm_reduce()
st.solve()
torch.cuda.synchronize()
buf = np.zeros(4 * 1024, dtype=np.uint64)
cnt = np.zeros(1, dtype=np.int64)
st.lib.gbm_debug_factime.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
assert st.lib.gbm_debug_factime(buf.ctypes.data, cnt.ctypes.data) == 0
k = int(min(cnt[0], 1024))
t = buf[: 4 * k].reshape(k, 4).astype(np.int64)
d = np.diff(t, axis=1) / 100.0
print(f"{k} syrk64 factor launches; median µs: tile {np.median(d[:, 0]):.2f} factor {np.median(d[:, 1]):.2f} "
      f"store {np.median(d[:, 2]):.2f}; max factor {d[:, 1].max():.2f}")
# fused panel tiles vs their launch's factor workgroup (times from that WG's entry, µs)
if hasattr(st.lib, "gbm_debug_paneltime"):
    pb = np.zeros(6 * 16384, dtype=np.uint64)
    pc = np.zeros(1, dtype=np.int64)
    st.lib.gbm_debug_paneltime.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    assert st.lib.gbm_debug_paneltime(pb.ctypes.data, pc.ctypes.data) == 0
    m = int(min(pc[0], 16384))
    P = pb[: 6 * m].reshape(m, 6).astype(np.int64)
    # factor records in launch order map to fk0 = 64, 128, ... for the syrk64 launches; match by order
    rows = []
    for fk in np.unique(P[:, 0]):
        sel = P[P[:, 0] == fk]
        e0 = sel[:, 1].min()
        rows.append(((sel[:, 2] - e0).mean() / 100, (sel[:, 3] - e0).mean() / 100, (sel[:, 3] - e0).max() / 100,
                     (sel[:, 4] - e0).max() / 100, len(sel)))
    r = np.array(rows)
    print(f"{len(r)} fused launches; mean over launches (µs from first panel-tile entry): tile done {r[:,0].mean():.2f} "
          f"wait end {r[:,1].mean():.2f} (max {r[:,2].mean():.2f}) last panel end {r[:,3].mean():.2f}; tiles/launch {r[:,4].mean():.1f}")
    print(f"factor WG (µs from its entry): tile {np.median(d[:, 0]):.2f} factor {np.median(d[:, 1]):.2f} store+publish {np.median(d[:, 2]):.2f}")
