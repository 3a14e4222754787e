"""Digest of everything a C2 stage-path fit returns (B, GEBVs, mu, msum) and the effects stage time, for builds
compared side by side (GBM_LIBGBM=...): fp64 stages, then the exact-GRM stages. Timing tool only."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gbm.sharded import HipExactShardStages, HipShardStages  # noqa: E402

n, p = (int(a) for a in sys.argv[1:3]) if len(sys.argv) > 2 else (5000, 50000)
lib = os.path.basename(os.environ.get("GBM_LIBGBM", "libgbm.so"))
y = np.random.default_rng(0).standard_normal(n)
for name, cls in (("fp64", HipShardStages), ("exact", HipExactShardStages)):
    st = cls(n, p, nrhs=1, lambda_=1.0, device=0)
    st.generate(4242, 0)
    st.load_phenotypes(y)
    ts = []
    for r in range(6):
        st.standardize()
        st.grm_syrk()
        st.grm_reduce()
        st.solve()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        st.effects()
        b.record()
        out = st.download()
        if r:
            ts.append(a.elapsed_time(b))
    h = hashlib.sha256()
    for k in ("B", "y_pred", "mu", "msum"):
        h.update(np.ascontiguousarray(out[k]).tobytes())
    print(f"{lib} {name} effects stage {np.median(ts):.4f} ms  digest {h.hexdigest()[:12]}", flush=True)
