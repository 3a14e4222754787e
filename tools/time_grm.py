"""Time the GRM SYRK launch alone (HIP events), for kernel variants loaded through GBM_LIBGBM."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
import torch  # noqa: E402

from gbm.sharded import HipShardStages  # noqa: E402

n, p = (int(a) for a in sys.argv[1:3]) if len(sys.argv) > 2 else (5000, 50000)
st = HipShardStages(n, p)
st.generate(4242, 0)
st.standardize()
for _ in range(2):
    st.grm_syrk()
ts = []
for _ in range(5):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    st.grm_syrk()
    b.record()
    b.synchronize()
    ts.append(a.elapsed_time(b))
ms = sorted(ts)[len(ts) // 2]
print(f"syrk {ms:.3f} ms  {n * (n + 1) * p / ms / 1e9:.1f} TF/s  frac {n * (n + 1) * p / ms / 1e9 / 78.6:.3f}  all {['%.2f' % t for t in ts]}")
