"""Time the exact-integer GRM stage alone (gbm_dev_grm_exact_i8 through HipExactShardStages.grm_syrk: the prep
kernels and the int8 digit GEMM), HIP events, for builds / test knobs compared side by side. Timing tool only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
import torch  # noqa: E402
from gbm.sharded import HipExactShardStages  # noqa: E402

n, p = (int(a) for a in sys.argv[1:3]) if len(sys.argv) > 2 else (5000, 50000)
st = HipExactShardStages(n, p)
st.generate(4242, 0)
st.standardize()
for _ in range(2):
    st.grm_syrk()
ts = []
for _ in range(7):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    st.grm_syrk()
    b.record()
    b.synchronize()
    ts.append(a.elapsed_time(b))
ms = sorted(ts)[len(ts) // 2]
print(f"exact grm stage {ms:.3f} ms  all {['%.2f' % t for t in ts]}", flush=True)
