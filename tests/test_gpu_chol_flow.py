"""The dataflow factorisation (csrc/chol_flow.hip: one persistent launch, left-looking 64x64
tiles handed over between workgroups through write-through stores and per-tile flags) against
the oracle and against the launch-per-panel path it replaces in gbm_dev_gblup_solve.

GBM_CHOL_FLOW_MAX (re-read at every solve) selects the path: npad <= limit → dataflow."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(np.abs(np.asarray(b)).max(), 1e-300))


def _pair(n, p, t, seed, lam):
    """Two stage objects holding the same summed G, q and Y (GRM computed once)."""
    import torch

    from gbm.sharded import HipShardStages
    X = oracle.synth_genotypes(seed, n, p)
    Y = oracle.synth_phenotypes(X, seed + 1, ntraits=t)
    a = HipShardStages(n, p, nrhs=t, lambda_=lam, device=0)
    a.upload_genotypes(X)
    a.load_phenotypes(Y)
    a.standardize()
    a.grm_syrk()
    a.grm_reduce()
    b = HipShardStages(n, p, nrhs=t, lambda_=lam, device=0)
    b.G.copy_(a.G)
    b.q.copy_(a.q)
    b.Y.copy_(a.Y)
    torch.cuda.synchronize()
    return X, Y, a, b


@pytest.mark.parametrize("n,p,t,seed,lam", [
    (64, 500, 1, 3, 1.0),        # one diagonal tile + the bordered column: 3 tiles in all
    (200, 1000, 2, 42, 1.0),     # C1 shape
    (1030, 1400, 3, 7, 0.5),     # ragged n (npad 1152)
    (3000, 2000, 2, 11, 0.8),    # 48 tile rows
    (5000, 1500, 1, 19, 1.0),    # the C2 individual count (80 tile rows)
])
def test_flow_matches_oracle_and_panel_path(gbm_env, n, p, t, seed, lam):
    import torch
    X, Y, flow, panel = _pair(n, p, t, seed, lam)
    gbm_env.setenv("GBM_CHOL_FLOW_MAX", "1000000")
    flow.solve()
    gbm_env.setenv("GBM_CHOL_FLOW_MAX", "0")
    panel.solve()
    torch.cuda.synchronize()
    assert int(flow.info.item()) == 0 and int(panel.info.item()) == 0
    gf = flow.gebv[:, :n].cpu().numpy().T
    gp = panel.gebv[:, :n].cpu().numpy().T
    af = flow.A[:, :n].cpu().numpy()
    ap = panel.A[:, :n].cpu().numpy()
    # the two paths sum the same updates in a different grouping: rounding-level differences only
    assert rel(gf, gp) < 1e-11
    assert rel(af, ap) < 1e-9
    assert rel(flow.mu.cpu().numpy(), panel.mu.cpu().numpy()) < 1e-11
    ref = oracle.gblup_fit(X, Y, lam)
    assert rel(gf, ref["y_pred"]) < 1e-9
    assert rel(flow.mu.cpu().numpy(), ref["mu"]) < 1e-9


def test_flow_repeated_solves_bit_identical(gbm_env):
    """Each tile's updates are summed in k order in its own accumulators, whatever the schedule:
    repeated solves (different workgroup placement and timing) give identical bits."""
    import torch
    gbm_env.setenv("GBM_CHOL_FLOW_MAX", "1000000")
    X, Y, a, b = _pair(2100, 900, 2, 5, 1.0)
    G0 = a.G.clone()
    first = None
    for _ in range(6):
        a.G.copy_(G0)
        a.solve()
        torch.cuda.synchronize()
        assert int(a.info.item()) == 0
        cur = (a.gebv.clone(), a.A.clone(), a.mu.clone())
        if first is None:
            first = cur
        else:
            assert all(torch.equal(x, y) for x, y in zip(cur, first))


@pytest.mark.parametrize("bad", [0, 700, 1029])
def test_flow_reports_first_failing_pivot(gbm_env, bad):
    """A matrix that is not positive definite: the factorisation ends (no hang) and info is the
    first failing column + 1, as in the launch-per-panel path."""
    import torch
    _, _, a, b = _pair(1030, 300, 1, 9, 1.0)
    for st in (a, b):
        st.G.zero_()
        st.G[:st.npad, :st.npad].fill_diagonal_(1.0)
        st.G[bad, bad] = -5.0
        st.q.fill_(1)
    gbm_env.setenv("GBM_CHOL_FLOW_MAX", "1000000")
    a.solve()
    gbm_env.setenv("GBM_CHOL_FLOW_MAX", "0")
    b.solve()
    torch.cuda.synchronize()
    assert int(a.info.item()) == bad + 1
    assert int(b.info.item()) == bad + 1


@pytest.mark.parametrize("wgs", ["1", "2", "7"])
def test_flow_few_resident_workgroups_complete_bit_identical(gbm_env, wgs):
    """Deadlock freedom: the chain workgroup waits only for its row's diagonal partial
    and the assistant's neighbour partial, the assistant only for a partial, a tile of the previous
    row and the chain's previous step, and every worker wait targets the chain's earlier steps or a
    task dequeued earlier (the right neighbour precedes its diagonal tile), so the launch completes
    with any number of resident workers — GBM_CHOL_FLOW_WGS caps them, down to one worker running
    every tile task in dequeue order beside the chain and the assistant — and gives the bits of the
    full-grid launch."""
    import torch
    gbm_env.setenv("GBM_CHOL_FLOW_MAX", "1000000")
    X, Y, a, b = _pair(1030, 700, 2, 13, 0.9)
    a.solve()
    gbm_env.setenv("GBM_CHOL_FLOW_WGS", wgs)
    b.solve()
    torch.cuda.synchronize()
    assert int(a.info.item()) == 0 and int(b.info.item()) == 0
    assert torch.equal(a.gebv, b.gebv) and torch.equal(a.A, b.A) and torch.equal(a.mu, b.mu)


@pytest.mark.parametrize("order,wgs", [("6", None), ("6", "1"), ("4", None)])
def test_flow_dequeue_orders_bit_identical(gbm_env, order, wgs):
    """The A/B dequeue orders (GBM_CHOL_FLOW_ORDER: 6 = the "other" tiles in pairs, one k-loop for two tiles;
    4 = round 4's order) sum every tile's updates in the same k order as the default: identical bits, also
    with a single worker running the paired order."""
    import torch
    gbm_env.setenv("GBM_CHOL_FLOW_MAX", "1000000")
    X, Y, a, b = _pair(3000, 700, 2, 21, 0.9)
    a.solve()
    gbm_env.setenv("GBM_CHOL_FLOW_ORDER", order)
    if wgs:
        gbm_env.setenv("GBM_CHOL_FLOW_WGS", wgs)
    b.solve()
    torch.cuda.synchronize()
    assert int(a.info.item()) == 0 and int(b.info.item()) == 0
    assert torch.equal(a.gebv, b.gebv) and torch.equal(a.A, b.A) and torch.equal(a.mu, b.mu)


def test_flow_timed_out_wait_drains_and_fails_loudly(gbm_env):
    """A wait that times out (info = −1; a bug guard, forced here by GBM_TEST_CHOL_FLOW_ABORT) stops
    the chain before it publishes another tile and keeps workers from taking new tasks:
    the launch drains at once and the solve reports info = −1 instead of computing on stale tiles.
    The next solve on the same buffers is clean."""
    import time

    import torch
    gbm_env.setenv("GBM_CHOL_FLOW_MAX", "1000000")
    X, Y, a, b = _pair(3000, 700, 1, 23, 1.0)
    gbm_env.setenv("GBM_TEST_CHOL_FLOW_ABORT", "1")
    t0 = time.perf_counter()
    a.solve()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert int(a.info.item()) == -1
    assert dt < 2.0, dt  # drained, not ~1 s per stuck wait
    gbm_env.delenv("GBM_TEST_CHOL_FLOW_ABORT")
    b.solve()
    torch.cuda.synchronize()
    assert int(b.info.item()) == 0
    ref = oracle.gblup_fit(X, Y, 1.0)
    assert rel(b.gebv[0, :3000].cpu().numpy(), ref["y_pred"][:, 0]) < 1e-9
