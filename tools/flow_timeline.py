"""Timeline of the dataflow factorisation (GBM_CHOL_FLOW_TRACE=1): where the chain through the
diagonal tiles spends its time. Timing tool only. N (default 5000)."""
import ctypes
import os
import sys

os.environ["GBM_CHOL_FLOW_TRACE"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gbm.sharded import HipShardStages  # noqa: E402

n = int(os.environ.get("N", "5000"))
st = HipShardStages(n, 2000, nrhs=1, lambda_=1.0, device=0)
st.generate(4242, 0)
st.load_phenotypes(np.random.default_rng(0).standard_normal(n))
st.standardize()
st.grm_syrk()
st.grm_reduce()
G0 = st.G.clone()
for _ in range(3):
    st.G.copy_(G0)
    st.solve()
torch.cuda.synchronize()
lib = st.lib
lib.gbm_debug_chol_flow_trace.restype = ctypes.c_int64
lib.gbm_debug_chol_flow_trace.argtypes = [ctypes.c_void_p, ctypes.c_int64]
nbc = (st.npad + 64) // 64
cap = nbc * (nbc + 1) // 2
buf = np.zeros((cap, 24), dtype=np.int64)
got = lib.gbm_debug_chol_flow_trace(buf.ctypes.data, cap)
assert got == cap, got
T = buf.astype(np.float64)
t0 = T[:, 3].min()
rec = {(int(r[0]), int(r[1])): r for r in T}
nb = nbc - 1
span = (T[:, 8].max() - t0) / 100.0
print(f"n={n} tiles={cap} span {span:.1f} us  ({span / nb:.1f} us per tile row)")
# record: i, j, id, start(3), k-loop end(4), tile in LDS(5), factor done / diag seen(6), stores issued(7), published(8)
D = np.array([rec[(i, i)] for i in range(nb)])
Nb = np.array([rec[(i, i + 1)] for i in range(nb)])
us = lambda a: a / 100.0
f = lambda a: f"mean {np.mean(a):6.2f} med {np.median(a):6.2f} max {np.max(a):6.2f}"
print("diag factor (k-end -> factored)        ", f(us(D[:, 6] - D[:, 4])))
print("diag Ld + partial + solve + publish    ", f(us(D[:, 8] - D[:, 6])))
print("partial ready before factor done (slack)", f(us(D[:, 6] - Nb[:, 8])))
print("diag published -> next diag k-end      ", f(us(D[1:, 4] - D[:-1, 8])))
print("next diag start before that hand-off   ", f(us(D[:-1, 8] - D[1:, 3])))
# factor internals (wave 0's timestamps): leaf steps end 9..12, leaf update end 13..15
st = [D[:, 5]] + [None] * 0
prev = D[:, 5]
for kb in range(4):
    print(f"  leaf {kb} steps                         ", f(us(D[:, 9 + kb] - prev)))
    if kb < 3:
        print(f"  leaf {kb} store+MFMA update+barriers  ", f(us(D[:, 13 + kb] - D[:, 9 + kb])))
        prev = D[:, 13 + kb]
print("  after last leaf -> factored            ", f(us(D[:, 6] - D[:, 12])))
print("  factored -> partial seen              ", f(us(D[:, 16] - D[:, 6])))
print("  partial seen -> in LDS (Ld issued)    ", f(us(D[:, 17] - D[:, 16])))
print("  neighbour solve                       ", f(us(D[:, 18] - D[:, 17])))
print("  store issue                           ", f(us(D[:, 7] - D[:, 18])))
print("  drain + flags                         ", f(us(D[:, 8] - D[:, 7])))
O = np.array([r for r in T if int(r[1]) > int(r[0]) + 1 and int(r[0]) < nb])
print("other tiles: diag seen -> published    ", f(us(O[:, 8] - O[:, 6])))
for i in (1, 10, 20, 40, 60, nb - 2):
    if i < nb:
        d = rec[(i, i)]
        print(f"  row {i}: diag start {us(d[3] - t0):8.1f} kend {us(d[4] - t0):8.1f} pub {us(d[8] - t0):8.1f}")
busy = (T[:, 8] - T[:, 3]).sum() / 100
print(f"task-time sum {busy:.0f} us over {span:.0f} us span")
