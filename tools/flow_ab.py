"""A/B of dataflow-Cholesky builds (GBM_LIBGBM=variants/libgbm_<name>.so): the solve stage time at each n and
a hash of everything the solve leaves (the factored G, the GEBVs, μ̂), so that variants meant to be
bit-identical can be checked against each other. Prints one JSON line per n. Timing tool only.
NS (default "5000,1500,9000"), REPS (default 10)."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gbm.sharded import HipShardStages  # noqa: E402

reps = int(os.environ.get("REPS", "10"))
for n in [int(v) for v in os.environ.get("NS", "5000,1500,9000").split(",")]:
    st = HipShardStages(n, 2000, nrhs=1, lambda_=1.0, device=0)
    st.generate(4242, 0)
    st.load_phenotypes(np.random.default_rng(0).standard_normal(n))
    st.standardize()
    st.grm_syrk()
    st.grm_reduce()
    G0 = st.G.clone()
    torch.cuda.synchronize()
    ts, digests = [], set()
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
        h = hashlib.sha256()
        for t in (st.G, st.gebv, st.mu):
            h.update(t.detach().cpu().numpy().tobytes())
        digests.add(h.hexdigest()[:16])
    print(json.dumps({"lib": os.path.basename(os.environ.get("GBM_LIBGBM", "libgbm.so")), "n": n,
                      "solve_ms_mean": round(float(np.mean(ts)), 4), "solve_ms_min": round(float(np.min(ts)), 4),
                      "info": int(st.info.item()), "digests": sorted(digests)}), flush=True)
    del st, G0
    torch.cuda.empty_cache()
