import sys, os
sys.path.insert(0, "genomicbreedingmodels.jl_amd"); sys.path.insert(0, "oracle")
import numpy as np, torch, oracle, gbm
from gbm.sharded import HipShardStages
n, p = 2000, 8000
X = oracle.synth_genotypes(p + 5, n, p)
outs = []
for overlap in (True, False):
    st = HipShardStages(n, p, nrhs=1, lambda_=1.0, device=0)
    st.upload_genotypes(X)
    if overlap:
        st.standardize_head(); print("j_from", st._j_from); st.grm_syrk_overlapped()
    else:
        st.standardize(); st.grm_syrk()
    st.grm_reduce(); torch.cuda.synchronize()
    outs.append([st.Z.clone(), st.mean.clone(), st.sd.clone(), st.keep.clone(), st.q.clone()])
for name, x, y in zip(["Z","mean","sd","keep","q"], outs[0], outs[1]):
    d = (x.double() - y.double()).abs()
    bad = torch.nonzero(d.reshape(d.shape[0], -1).amax(dim=1) if d.dim() > 1 else d).flatten()
    print(name, "equal" if torch.equal(x, y) else f"DIFF max {d.max().item():.3e} rows {bad[:5].tolist()} ... n_bad {bad.numel()}")
