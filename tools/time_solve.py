"""Time the GBLUP solve stage alone (n = 5000 by default) on the device-level ABI.
Run under rocprofv3 --kernel-trace --stats for per-kernel times. Timing tool only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
import torch  # noqa: E402
from gbm.sharded import HipShardStages  # noqa: E402

n = int(os.environ.get("N", "5000"))
p = int(os.environ.get("P", "4000"))
reps = int(os.environ.get("REPS", "5"))
st = HipShardStages(n, p, nrhs=1, lambda_=1.0, device=0)
st.generate(4242, 0)
import numpy as np  # noqa: E402
st.load_phenotypes(np.random.default_rng(0).standard_normal(n))
st.standardize()
st.grm_syrk()
st.grm_reduce()
G0 = st.G.clone()
torch.cuda.synchronize()
ts = []
for r in range(reps + 1):
    st.G.copy_(G0)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    st.solve()
    e1.record()
    torch.cuda.synchronize()
    if r:
        ts.append(e0.elapsed_time(e1))
print(f"solve n={n}: {np.mean(ts):.3f} ms (min {np.min(ts):.3f}) flow_max={os.environ.get('GBM_CHOL_FLOW_MAX', 'default')} info={int(st.info.item())}")
