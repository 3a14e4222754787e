"""Phase timeline of one BRR Gibbs iteration's 128-marker launches (workgroup 0), from a libgbm
variant built with -DBRR_TL (tools/build_variant.sh brrtl -DBRR_TL). Analysis tool only."""
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
# s_memtime slots (shader clock): 0 entry(w3) 2 r~ formed(w3) 3 M rows in regs(w0) 4 after barrier 1
# 5 after GEMV barrier 6 e updated 7 Xb landed + sync 8 partials stored ; memrealtime (100 MHz): 1 entry 9 end
base = t[:, 0]
names = {11: "w0 before row loads", 12: "w0 row loads issued", 10: "w3 partial loads issued", 2: "r~ formed (w3)", 3: "M rows loaded (w0)", 4: "barrier 1", 5: "GEMV+barrier 2", 6: "e updated",
         7: "Xb landed+sync", 8: "partials stored"}
sl = slice(5, nb - 5)
clk = np.median((t[sl, 8] - t[sl, 0]) / np.maximum(t[sl, 9] - t[sl, 1], 1)) * 100.0  # MHz
print(f"shader clock ~{clk:.0f} MHz")
for k, nm in names.items():
    v = (t[sl, k] - base[sl]) / clk
    print(f"{nm:22s} median {np.median(v):7.2f} us  p10 {np.percentile(v, 10):7.2f}  p90 {np.percentile(v, 90):7.2f}")
dur = (t[sl, 9] - t[sl, 1]) / 100.0
gap = (t[6:nb - 4, 1] - t[5:nb - 5, 9]) / 100.0
print(f"WG0 entry->end median {np.median(dur):.2f} us; end(k) -> entry(k+1) median {np.median(gap):.2f} us")
