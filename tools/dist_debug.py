"""Where a distributed factorisation differs from the redundant one (debug tool): the upper factor,
the lower copy and the diagonal-block factors, per 64-block. Usage: python tools/dist_debug.py R n"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from gbm.sharded import HipShardStages, chol_distributed  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1500
tail = int(sys.argv[3]) if len(sys.argv) > 3 else 256
os.environ.update(GBM_CHOL_G4_LIM="0", GBM_CHOL_G8_LIM="-1", GBM_CHOL_G16_LIM="-1", GBM_UPD64_LIM="128",
                  GBM_CHOL_FLOW_MAX="0")
X = oracle.synth_genotypes(n + R, n, 1200)
Y = oracle.synth_phenotypes(X, 3, ntraits=2)
sts = [HipShardStages(n, 1200, nrhs=2, lambda_=0.8, device=0) for _ in range(R + 1)]
sts[0].upload_genotypes(X)
sts[0].load_phenotypes(Y)
sts[0].standardize()
sts[0].grm_syrk()
sts[0].grm_reduce()
for st in sts[1:]:
    st.G.copy_(sts[0].G)
    st.q.copy_(sts[0].q)
    st.Y.copy_(sts[0].Y)
torch.cuda.synchronize()
ref = sts[0]
ref.solve()
for ov in ("0", "1"):
    os.environ["GBM_DIST_OVERLAP"] = ov
    for st in sts[1:]:
        st.G.copy_(sts[1].G if False else sts[0].G)
    # restart from the summed G: re-run the GRM copy
    G0 = torch.empty_like(ref.G)
    sts[1].G.zero_()
    ranks = sts[1:]
    src = HipShardStages(n, 1200, nrhs=2, lambda_=0.8, device=0)
    src.upload_genotypes(X)
    src.load_phenotypes(Y)
    src.standardize()
    src.grm_syrk()
    src.grm_reduce()
    for st in ranks:
        st.G.copy_(src.G)
    torch.cuda.synchronize()

    def allgather(packs):
        g = torch.cat(packs)
        return [g] * len(packs)

    chol_distributed(ranks, list(range(R)), R, allgather, tail_rows=tail)
    torch.cuda.synchronize()
    npad = ref.npad
    Gr = ref.G.cpu().numpy()
    for k, st in enumerate(ranks):
        Gd = st.G.cpu().numpy()
        up = np.triu(np.ones((npad, npad), bool), 1)
        lo = np.tril(np.ones((npad, npad), bool), -1)
        dU = (Gr[:npad, :npad] != Gd[:npad, :npad]) & up
        dL = (Gr[:npad, :npad] != Gd[:npad, :npad]) & lo
        dD = np.diag(Gr[:npad, :npad]) != np.diag(Gd[:npad, :npad])
        dR = Gr[:npad, npad:] != Gd[:npad, npad:]
        wsr = ref.ws_solve.cpu().numpy()
        wsd = st.ws_solve.cpu().numpy()
        Ldn = npad * 64 * 8
        print(f"overlap={ov} rank {k}: upper diffs {dU.sum()}, lower {dL.sum()}, diag {dD.sum()}, rhs {dR.sum()}, "
              f"Ld bytes diff {(wsr[:Ldn] != wsd[:Ldn]).sum()}, A equal {torch.equal(st.A, ref.A)}")
        for name, d in (("upper", dU), ("lower", dL)):
            if d.any():
                bi = np.argwhere(d)
                blk = sorted(set((int(i) // 64, int(j) // 64) for i, j in bi[:200000]))
                print(f"  {name}: first {bi[0].tolist()}, 64-blocks (first 20): {blk[:20]}")
        if dR.any():
            print("  rhs first", np.argwhere(dR)[0].tolist())
