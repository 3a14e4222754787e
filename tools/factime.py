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
