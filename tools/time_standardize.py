"""Time the standardisation stage alone (gbm_dev_standardize through HipShardStages.standardize, C2 shape by
default), HIP events, with a digest of Z / mean / sd, for builds compared side by side (GBM_LIBGBM=...).
Timing tool only."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
import torch  # noqa: E402
from gbm.sharded import HipShardStages  # noqa: E402

n, p = (int(a) for a in sys.argv[1:3]) if len(sys.argv) > 2 else (5000, 50000)
st = HipShardStages(n, p, nrhs=1, lambda_=1.0, device=0)
st.generate(4242, 0)
for _ in range(2):
    st.standardize()
ts = []
for _ in range(15):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    st.standardize()
    b.record()
    b.synchronize()
    ts.append(a.elapsed_time(b))
h = hashlib.sha256()
for t in (st.Z, st.mean, st.sd):
    h.update(t.cpu().numpy().tobytes())
ms = sorted(ts)[len(ts) // 2]
lib = os.path.basename(os.environ.get("GBM_LIBGBM", "libgbm.so"))
print(f"{lib} standardize {ms:.4f} ms  min {min(ts):.4f}  digest {h.hexdigest()[:12]}", flush=True)
