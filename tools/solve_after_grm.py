"""Time the GBLUP solve stage (gbm_dev_gblup_solve) on a G built by the fp64 GRM and on one built by the exact
int8 GRM, same n, same process, alternating, HIP events; optionally right after a fresh GRM (AFTER=1) so the
solve runs with the GRM's clocks and cache state, as in the step. Timing tool only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gbm.sharded import HipExactShardStages, HipShardStages  # noqa: E402

n, p = int(os.environ.get("N", "5000")), int(os.environ.get("P", "50000"))
after = os.environ.get("AFTER", "0") == "1"
# between the GRM and the solve (AFTER=1): "touch" = G copied out and back (G last written, as after the fp64
# reduce), "idle" = the GPU spins ≈ 2 ms in a one-wave kernel (clocks settle), "" = nothing
between = os.environ.get("BETWEEN", "")
y = np.random.default_rng(0).standard_normal(n)
stages = {}
for name, cls in (("fp64", HipShardStages), ("exact", HipExactShardStages)):
    st = cls(n, p, nrhs=1, lambda_=1.0, device=0)
    st.generate(4242, 0)
    st.load_phenotypes(y)
    st.standardize()
    st.grm_syrk()
    st.grm_reduce()
    stages[name] = (st, st.G.clone())
torch.cuda.synchronize()
res = {k: [] for k in stages}
for r in range(7):
    for name, (st, G0) in stages.items():
        if after:
            st.grm_syrk()
            st.grm_reduce()
            if between == "touch":
                tmp = st.G.clone()
                st.G.copy_(tmp)
                del tmp
            elif between == "idle":
                torch.cuda._sleep(5_000_000)
        else:
            st.G.copy_(G0)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        st.solve()
        b.record()
        b.synchronize()
        if r:
            res[name].append(a.elapsed_time(b))
for name, ts in res.items():
    print(f"{name:6s} after_grm={int(after)} {between:5s} solve median {np.median(ts):.3f} ms  {['%.3f' % t for t in ts]}", flush=True)
