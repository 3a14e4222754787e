"""Phase timeline of one BRR Gibbs iteration's 128-marker launches (workgroup 0), from a libgbm
built with -DBRRX_TL (temporary instrumentation). Analysis tool only."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
import gbm
from gbm import synth
n, p = 10000, 20000
X = synth.genotypes(4242, n, p)
y = synth.qtl_phenotypes(4242, n, p, 1)[:, 0]
gbm.brr_arrays(X, y, n_iter=3, n_burnin=1, thin=1)
lib = gbm.load_library()
buf = np.zeros(16 * 1024, dtype=np.uint64)
assert lib.gbm_debug_brrtl(ctypes.c_void_p(buf.ctypes.data)) == 0
t = buf.reshape(1024, 16).astype(np.int64)
nb = (p + 127) // 128
t = t[:nb]
# wave 0: [0] entry [1] after sync1 [2] A done [3] after sync3 ; wave 1: [4] e update done [5] end
base = t[:, 0]
ph = {"sync1": t[:, 1] - base, "A_done": t[:, 2] - base, "B_start": t[:, 3] - base, "e_upd(w1)": t[:, 4] - base,
      "end(w1)": t[:, 5] - base, "next_entry": np.r_[t[1:, 0] - t[:-1, 0], 0]}
for k, v in ph.items():
    print(f"{k:12s} median {np.median(v[5:-5]) / 2.4e3:7.2f} us (cycles {np.median(v[5:-5]):.0f})")
