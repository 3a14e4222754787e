"""Phase timeline of one BRR sweep (brr_sweep128_kernel, workgroup 0, per 128-marker block), from
a libgbm variant built with -DBRR_TL (the instrumented kernel is kept in variants/). Analysis
tool only."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
import gbm
from gbm import synth
n, p = int(sys.argv[1]) if len(sys.argv) > 1 else 10000, 100000
X = synth.genotypes(4242, n, p)
y = synth.qtl_phenotypes(4242, n, p, 1)[:, 0]
gbm.brr_arrays(X, y, n_iter=3, n_burnin=1, thin=1)
lib = gbm.load_library()
buf = np.zeros(2048 * 16, dtype=np.uint64)
assert lib.gbm_debug_brrtl(ctypes.c_void_p(buf.ctypes.data)) == 0
nb = (p + 127) // 128
t = buf.reshape(2048, 16).astype(np.int64)[:nb]
clk = 2400.0  # MHz (s_memtime: shader clock)
names = {1: "poll done (w3)", 2: "r~ formed (w3)", 3: "barrier 1 (w0)", 4: "GEMV + barrier 2", 5: "e updated",
         6: "es barrier", 7: "published (w3)"}
sl = slice(5, nb - 5)
base = t[sl, 0]
for k, nm in names.items():
    v = (t[sl, k] - base) / clk
    print(f"{nm:20s} median {np.median(v):7.2f} us  p10 {np.percentile(v, 10):7.2f}  p90 {np.percentile(v, 90):7.2f}")
per = (t[6:nb - 4, 0] - t[5:nb - 5, 0]) / clk
print(f"block-to-block (poll start) median {np.median(per):.2f} us")
