"""The distributed GBLUP factorisation (gbm.sharded.chol_distributed over the gbm_dev_chol_* ABI)
rehearsed in one process: R ranks, each a full copy of the summed G on the one GPU, each updating
only its own 128-column tiles; the all-gathers are concatenations (the area exchange on the side
stream unless GBM_DIST_OVERLAP = 0). The factorisation must be
bit-identical to the redundant single-rank solve (the same kernel computes every tile) and match
the oracle. Panel-group thresholds are forced so that 16/8/4/2-panel groups and the single-panel
tail all occur at test size."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(np.abs(np.asarray(b)).max(), 1e-300))


def _stages(R, X, Y, lam):
    import torch

    from gbm.sharded import HipShardStages
    n, p = X.shape
    sts = [HipShardStages(n, p, nrhs=Y.shape[1], lambda_=lam, device=0) for _ in range(R + 1)]
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
    return sts[0], sts[1:]


@pytest.mark.parametrize("R,n,lims,tail", [
    (2, 1500, ("0", "-1", "-1"), 256),     # 4-panel groups
    (3, 1500, ("0", "-1", "-1"), 0),       # 4-panel groups down to the 2-panel / single-panel tail
    (8, 3000, ("0", "0", "0"), 0),         # 16, 8, 4, 2-panel groups, then single panels
    (4, 1030, ("0", "0", "0"), 512),       # ragged n, early switch to the redundant tail
    (8, 3000, ("0", "0", "0"), "0-seq"),   # as above without the side-stream area exchange
    (8, 3000, ("0", "0", "0"), "0-chain"),  # the panel phase as panel / row-update launches, not one group launch
    (8, 3000, ("0", "0", "0"), "0-nolook"),  # the next group's panels after the whole trailing update (no look-ahead)
    (8, 3000, ("0", "0", "0"), "0-tailflow"),  # the last 1024 rows in one dataflow launch (GBM_CHOL_TAIL_FLOW)
])
def test_distributed_factorisation_bit_identical(gbm_env, R, n, lims, tail):
    import torch

    from gbm.sharded import chol_distributed
    gbm_env.setenv("GBM_CHOL_G4_LIM", lims[0])
    gbm_env.setenv("GBM_CHOL_G8_LIM", lims[1])
    gbm_env.setenv("GBM_CHOL_G16_LIM", lims[2])
    gbm_env.setenv("GBM_UPD64_LIM", "128")
    gbm_env.setenv("GBM_CHOL_FLOW_MAX", "0")  # reference: the redundant launch-per-panel solve
    if isinstance(tail, str):  # "<rows>-seq" / "-chain" / "-nolook": GBM_DIST_OVERLAP / GBM_CHOL_GROUP_KERNEL /
        # GBM_DIST_LOOKAHEAD = 0; "-tailflow": GBM_CHOL_TAIL_FLOW = 1024
        var = {"seq": "GBM_DIST_OVERLAP", "chain": "GBM_CHOL_GROUP_KERNEL", "nolook": "GBM_DIST_LOOKAHEAD",
               "tailflow": "GBM_CHOL_TAIL_FLOW"}
        gbm_env.setenv(var[tail.split("-")[1]], "1024" if tail.endswith("tailflow") else "0")
        tail = int(tail.split("-")[0])
    X = oracle.synth_genotypes(n + R, n, 1200)
    Y = oracle.synth_phenotypes(X, 3, ntraits=2)
    ref_st, ranks = _stages(R, X, Y, 0.8)
    ref_st.solve()

    def allgather(packs):
        g = torch.cat(packs)
        return [g] * len(packs)

    chol_distributed(ranks, list(range(R)), R, allgather, tail_rows=tail)
    torch.cuda.synchronize()
    for st in ranks:
        assert int(st.info.item()) == 0
        assert torch.equal(st.A, ref_st.A) and torch.equal(st.gebv, ref_st.gebv) and torch.equal(st.mu, ref_st.mu)
    ref = oracle.gblup_fit(X, Y, 0.8)
    assert rel(ranks[0].gebv[:, :n].cpu().numpy().T, ref["y_pred"]) < 1e-9
