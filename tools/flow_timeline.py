"""Timeline of the dataflow factorisation (GBM_CHOL_FLOW_TRACE=1): where the chain workgroup's steps
spend their time, and how far ahead of it the partials it needs arrive. Timing tool only.
N (default 5000)."""
import ctypes
import os
import sys

os.environ.setdefault("GBM_CHOL_FLOW_TRACE", "1")
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
torch.cuda.synchronize()
print("GRM done", file=sys.stderr, flush=True)
for r in range(3):
    st.G.copy_(G0)
    st.solve()
    torch.cuda.synchronize()
    print(f"traced solve {r} done, info={int(st.info.item())}", file=sys.stderr, flush=True)
lib = st.lib
lib.gbm_debug_chol_flow_trace.restype = ctypes.c_int64
lib.gbm_debug_chol_flow_trace.argtypes = [ctypes.c_void_p, ctypes.c_int64]
nbc = (st.npad + 64) // 64
ntasks = nbc * (nbc + 1) // 2
nb = nbc - 1
cap = ntasks + nbc
buf = np.zeros((cap, 32), dtype=np.int64)  # kTraceRec
got = lib.gbm_debug_chol_flow_trace(buf.ctypes.data, cap)
assert got == cap, got
T = buf.astype(np.float64)
if os.environ.get("FLOW_DUMP"):  # raw records for offline analysis
    np.save(os.environ["FLOW_DUMP"], buf)
W = T[:ntasks]
Ch = T[ntasks:ntasks + nb]  # chain step i: o[3 + e] = ct[e]
ct = Ch[:, 3:19]
t0 = min(W[W[:, 3] > 0, 3].min(), ct[:, 0].min())
us = lambda a: a / 100.0
f = lambda a: f"mean {np.mean(a):6.2f} med {np.median(a):6.2f} max {np.max(a):6.2f}"
span = (max(W[:, 8].max(), ct[:, 12].max()) - t0) / 100.0
print(f"n={n} tiles={ntasks} span {span:.1f} us  ({span / nb:.1f} us per tile row)")
step = np.diff(ct[:, 0])
print("chain step (start -> next start)        ", f(us(step)))
print("  factor (start -> factored)             ", f(us(ct[:, 8] - ct[:, 0])))
prev = ct[:, 0]
for kb in range(4):  # wave kb owns leaf kb; the next leaf's owner goes on as soon as it ends
    print(f"    leaf {kb} (start / previous leaf end -> end)", f(us(ct[:, 1 + kb] - prev)))
    own0 = ct[:, 13] if kb == 0 else ct[:, 4 + kb]
    print(f"      leaf {kb}: hand-over (-> own start)   ", f(us(own0 - prev)))
    print(f"      leaf {kb}: own 16 steps               ", f(us(ct[:, 1 + kb] - own0)))
    prev = ct[:, 1 + kb]
if (Ch[1:, 24:28] > 0).all():  # wave 1's hand-over into leaf 1 (steps >= 1: with the previous step's update)
    w1 = Ch[1:, 24:28]
    l0 = ct[1:, 1]
    print("      wave 1: (1,2)/(1,3) waits begin, from leaf 0 end", f(us(w1[:, 0] - l0)))
    print("      wave 1: waits end, from leaf 0 end           ", f(us(w1[:, 1] - l0)))
    print("      wave 1: last row group's MFMAs issued, from leaf 0 end", f(us(w1[:, 2] - l0)))
    print("      wave 1: rows read back, from leaf 0 end      ", f(us(w1[:, 3] - l0)))
print("    last leaf end -> factored (sync)     ", f(us(ct[:, 8] - ct[:, 4])))
print("    X2 (neighbour partial) in LDS, from start", f(us(ct[:, 9] - ct[:, 0])))
print("    Xn (next diag partial) in LDS, from start", f(us(ct[:, 14] - ct[:, 0])))
print("    helper block rows done, from start   ", f(us(ct[:, 15] - ct[:, 0])))
if (Ch[:, 22] > 0).all():
    print("      wave 0 (column blocks 0, 3), from start", f(us(Ch[:, 22] - ct[:, 0])))
    print("      wave 2 (column block 2), from start  ", f(us(Ch[:, 23] - ct[:, 0])))
print("  neighbour solve + Ld stores            ", f(us(ct[:, 10] - ct[:, 8])))
print("  next tile update (k = i)               ", f(us(ct[:, 11] - ct[:, 10])))
print("  drain + flags                          ", f(us(ct[:, 12] - ct[:, 11])))
print("  published -> next step start           ", f(us(ct[1:, 0] - ct[:-1, 12])))
A = Ch[1:, 19:22]  # the assistant's step i >= 1: partial + U_i-1,i+1 ready, U_i-1,i seen, published
if (A > 0).all():
    st1 = ct[1:, 0]
    print("assistant: partial and U(i-1,i+1) ready, from start", f(us(A[:, 0] - st1)))
    print("assistant: U(i-1,i) (chain) seen, from start       ", f(us(A[:, 1] - st1)))
    print("assistant: published, from start                   ", f(us(A[:, 2] - st1)))
rec = {(int(r[0]), int(r[1])): r for r in W if r[8] > 0}
if (A > 0).all():  # the assistant's input U(i-1,i+1): when its worker dequeued, finished k, saw the leaves, published
    T2 = np.array([rec[(i - 1, i + 1)] for i in range(1, nb) if (i - 1, i + 1) in rec])
    if len(T2) == nb - 1:
        st1 = ct[1:, 0]
        for name, col in (("dequeued", 3), ("k-loop done", 4), ("last leaf seen", 6), ("published", 8)):
            print(f"U(i-1,i+1) worker {name:15s}, from step i start", f(us(T2[:, col] - st1)))
    T3 = np.array([rec[(i, i + 1)] for i in range(1, nb)])
    for name, col in (("dequeued", 3), ("k-loop done", 4), ("published", 8)):
        print(f"partial (i,i+1) worker {name:11s}, from step i start", f(us(T3[:, col] - st1)))
    T4 = np.array([rec[(i - 2, i + 1)] for i in range(2, nb)])
    print("U(i-2,i+1) published, from step i start     ", f(us(T4[:, 8] - st1[1:])))
    T5 = np.array([rec[(i - 2, i)] for i in range(2, nb)])
    print("U(i-2,i) published, from step i start       ", f(us(T5[:, 8] - st1[1:])))
# partial readiness: neighbour (i, i+1) and diagonal (i+1, i+1) published vs the chain's need
nbp = np.array([rec[(i, i + 1)][8] for i in range(nb)])
dgp = np.array([rec[(i, i)][8] for i in range(1, nb)])
print("neighbour partial published before factored", f(us(ct[:, 8] - nbp)))
print("diag partial published before needed     ", f(us(ct[:-1, 8] - dgp)))
O = np.array([r for r in W if int(r[1]) > int(r[0]) + 1 and int(r[0]) < nb and r[8] > 0])
print("other tiles: last leaf seen -> published  ", f(us(O[:, 8] - O[:, 6])))
busy = (W[:, 8] - W[:, 3]).clip(0).sum() / 100
print(f"worker task-time sum {busy:.0f} us over {span:.0f} us span")
