"""HIP path vs the CPU oracle (numpy/LAPACK restatement) — the parity tests proper.

Tolerance (north_star): GEBVs within 1e-6 relative in fp64; b_hat within 1e-6 relative to
max|b|. In practice the fp64 MFMA path agrees to ~1e-12 at these sizes, and we assert 1e-9 on
y_pred as a tighter regression guard (still far inside the contract)."""
import numpy as np
import pytest

import oracle
import gbm

pytestmark = pytest.mark.gpu

TOL_CONTRACT = 1e-6
TOL_TIGHT = 1e-9


def rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(np.abs(np.asarray(b)).max(), 1e-300))


@pytest.mark.parametrize("n,p,t,seed", [
    (200, 1000, 1, 42),      # config C1 shape
    (333, 1777, 3, 7),       # ragged: n, p not tile multiples; 3 traits
    (129, 64, 1, 3),         # p < n (G rank deficient; λ keeps V SPD)
    (64, 5000, 2, 5),        # single tile, many loci
    (1000, 3000, 1, 11),     # several Cholesky panels
])
def test_gblup_matches_oracle(n, p, t, seed):
    X = oracle.synth_genotypes(seed, n, p)
    Y = oracle.synth_phenotypes(X, seed + 1, ntraits=t)
    b_hat, y_pred, mu, q = gbm.gblup_arrays(X, Y, lambda_=1.0)
    ref = oracle.gblup_fit(X, Y, 1.0)
    assert q == ref["q"]
    assert rel(y_pred, ref["y_pred"]) < TOL_TIGHT
    assert rel(mu, ref["mu"]) < TOL_TIGHT
    assert rel(b_hat, ref["b_hat"]) < TOL_CONTRACT
    # predict-form identity (src/prediction.jl:228): b0 + X b reproduces the GEBVs
    assert rel(oracle.predict_linear(X, b_hat), y_pred) < TOL_TIGHT


@pytest.mark.parametrize("grm", ["fp64", "exact"])
@pytest.mark.parametrize("n,p", [(2, 40), (3, 1), (65, 2), (127, 1)])
def test_tiny_shapes_match_oracle(n, p, grm):
    """The smallest fits the reference accepts (≥ 2 entries, prediction.jl:117-123) and single-locus GRMs:
    one diagonal tile with mostly padding, p below one LDS stage of loci; both GRM modes."""
    rng = np.random.default_rng(n * 1000 + p)
    X = rng.integers(0, 3, size=(n, p)).astype(np.float64) / 2.0
    X[0, :], X[1, :] = 0.0, 1.0  # every locus polymorphic
    Y = rng.standard_normal((n, 2))
    b_hat, y_pred, mu, q = gbm.gblup_arrays(X, Y, lambda_=0.7, grm=grm)
    ref = oracle.gblup_fit(X, Y, 0.7)
    assert q == ref["q"] == p
    assert rel(y_pred, ref["y_pred"]) < TOL_TIGHT
    assert rel(mu, ref["mu"]) < TOL_TIGHT
    assert rel(b_hat, ref["b_hat"]) < TOL_CONTRACT


def test_monomorphic_and_lambda():
    n, p = 150, 400
    X = oracle.synth_genotypes(99, n, p)
    X[:, 5] = 0.0      # monomorphic (dropped, b = 0)
    X[:, 17] = 0.5     # monomorphic
    X[:, 399] = 1.0
    Y = oracle.synth_phenotypes(X, 3)
    for lam in (0.1, 1.0, 10.0):
        b_hat, y_pred, mu, q = gbm.gblup_arrays(X, Y, lambda_=lam)
        ref = oracle.gblup_fit(X, Y, lam)
        assert q == ref["q"] == p - 3
        assert b_hat[1 + 5, 0] == 0.0 and b_hat[1 + 17, 0] == 0.0 and b_hat[1 + 399, 0] == 0.0
        assert rel(y_pred, ref["y_pred"]) < TOL_TIGHT
        assert rel(b_hat, ref["b_hat"]) < TOL_CONTRACT


def test_grm_and_colstats_match_oracle():
    n, p = 257, 900
    X = oracle.synth_genotypes(5, n, p)
    X[:, 3] = 0.5
    G, q = gbm.grm(X)
    Gr, qr = oracle.grm(X)
    assert q == qr
    assert rel(G, Gr) < 1e-12
    assert np.array_equal(G, G.T)
    m, s, k, q2 = gbm.colstats(X)
    mr, sr, kr = oracle.colstats(X)
    assert q2 == qr and np.array_equal(k, kr)
    assert rel(m, mr) < 1e-14 and rel(s[k], sr[kr]) < 1e-13


@pytest.mark.parametrize("n,p,ploidy,devices", [
    (200, 1000, 2, None),
    (333, 1777, 4, None),     # ragged n and p (edge kernel), tetraploid frequencies k/4
    (1030, 900, 4, [0, 0]),   # two same-device loci shards summed on the device
])
def test_grm_ploidy_aware_matches_oracle(n, p, ploidy, devices):
    """gbm_grm_ploidy_aware (replaces Core's grmploidyaware at src/gwas.jl:117-121; the Core
    formula is un-vendored, so the pin is the oracle's VanRaden-for-ploidy-k restatement, parity
    unpinned): centred frequencies on the device, the MFMA GRM, scaled by k / Σ f(1 − f); ploidy
    inferred as the reference does (src/gwas.jl:119)."""
    rng = np.random.default_rng(n + p)
    X = np.round(rng.random((n, p)) ** 2 * ploidy) / ploidy  # frequencies k/ploidy, skewed
    X[:, 3] = 0.5                                              # a monomorphic column
    G, den = gbm.grm_ploidy_aware(X, devices=devices)
    ref, den_ref = oracle.grm_ploidy_aware(X, ploidy)
    assert gbm.infer_ploidy(X) == ploidy
    assert G.shape == (n, n) and abs(den - den_ref) <= 1e-12 * den_ref
    assert rel(G, ref) < 1e-12
    assert np.array_equal(G, G.T)


def test_dosage_i8_path_equals_f64_path():
    n, p, ploidy = 180, 700, 4
    rng = np.random.default_rng(1)
    D = np.asfortranarray(rng.integers(0, ploidy + 1, size=(n, p)).astype(np.int8))
    X = D.astype(np.float64) / ploidy
    Y = oracle.synth_phenotypes(X, 2, ntraits=2)
    lib = gbm.load_library()
    from gbm import _lib
    Yf = np.asfortranarray(Y)
    b_hat = np.zeros((p + 1, 2), order="F")
    y_pred = np.zeros((n, 2), order="F")
    mu = np.zeros(2)
    q = np.zeros(1, dtype=np.int64)
    rc = lib.gbm_gblup_fit_dosage_i8(_lib.ptr(D), n, p, n, ploidy, _lib.ptr(Yf), n, 2, 1.0, None, 0,
                                     _lib.ptr(b_hat), _lib.ptr(y_pred), _lib.ptr(mu), _lib.ptr(q))
    _lib.check(rc, "dosage")
    b2, y2, mu2, q2 = gbm.gblup_arrays(X, Y, 1.0)
    assert q[0] == q2
    assert np.array_equal(y_pred, y2) and np.array_equal(b_hat, b2)


def test_predict_gpu_matches_linear_predictor():
    n, p = 300, 1200
    X = oracle.synth_genotypes(21, n, p)
    Y = oracle.synth_phenotypes(X, 4)
    b_hat, y_pred, _, _ = gbm.gblup_arrays(X, Y)
    names = [f"e{i}" for i in range(n)]
    loci = [f"l{j}" for j in range(p)]
    genomes = gbm.Genomes(names, ["pop"] * n, loci, X)
    fit = gbm.Fit(n=n, l=p + 1, model="gblup", b_hat_labels=["intercept"] + loci, b_hat=b_hat[:, 0],
                  entries=names, populations=["pop"] * n, y_true=Y[:, 0], y_pred=y_pred[:, 0])
    out = gbm.predict(fit, genomes, np.arange(1, n + 1))
    assert rel(out, y_pred[:, 0]) < TOL_TIGHT


def test_errors_are_loud():
    X = oracle.synth_genotypes(1, 50, 100)
    with pytest.raises(gbm.ArgumentError):
        gbm.gblup_arrays(X, np.full(50, np.nan))
    with pytest.raises(gbm.GBMError):
        gbm.gblup_arrays(X, np.ones(50))  # zero variance
    with pytest.raises(gbm.GBMError):
        gbm.gblup_arrays(np.zeros((50, 10)), np.arange(50.0))  # no polymorphic locus
    with pytest.raises(gbm.ArgumentError):
        gbm.gblup_arrays(X, np.arange(50.0), lambda_=0.0)


def test_sharded_stages_single_rank_match_oracle():
    """The device-level stage API (as bench.py drives it) on one rank == the oracle, with the
    on-device genotype generator bit-identical to the oracle's."""
    import torch
    from gbm.sharded import HipShardStages, LocalComm, assemble_b_hat, sharded_gblup_step

    n, p, seed = 700, 2500, 77
    st = HipShardStages(n, p, nrhs=2, lambda_=1.0, device=0)
    st.generate(seed, 0)
    X = oracle.synth_genotypes(seed, n, p)
    Xd = st.X[:, :n].cpu().numpy().T
    assert np.array_equal(Xd, X)  # bit-exact generator
    assert torch.count_nonzero(st.X[:, n:]).item() == 0
    Y = oracle.synth_phenotypes(X, 3, ntraits=2)
    st.load_phenotypes(Y)
    out = sharded_gblup_step(st, LocalComm())
    out2 = sharded_gblup_step(st, LocalComm())  # steps are repeatable (X kept intact)
    ref = oracle.gblup_fit(X, Y, 1.0)
    assert rel(out["y_pred"], ref["y_pred"]) < TOL_TIGHT
    assert np.array_equal(out["y_pred"], out2["y_pred"])
    b_hat = assemble_b_hat(out["mu"], out["msum"], [out["B"]], p)
    assert rel(b_hat, ref["b_hat"]) < TOL_CONTRACT


@pytest.mark.parametrize("n,p", [
    (1030, 1234),   # ragged last tile column of 6: the GRM's edge workgroups
    (1088, 37),     # edge of exactly 64 columns; fewer loci than one MFMA k-block batch
    (1100, 2049),   # last column of 76: the ordinary (masked) tile path
    (4999, 600),    # C2-like ragged n (edge of 7), 10 loci-range partials
])
def test_grm_ragged_last_tile_column(n, p):
    X = oracle.synth_genotypes(n + p, n, p)
    G, q = gbm.grm(X)
    Gr, qr = oracle.grm(X)
    assert q == qr
    assert rel(G, Gr) < 1e-12
    assert np.array_equal(G, G.T)


def test_gblup_with_grm_edge_matches_oracle():
    n, p = 1030, 1500
    X = oracle.synth_genotypes(8, n, p)
    Y = oracle.synth_phenotypes(X, 9, ntraits=2)
    b_hat, y_pred, mu, q = gbm.gblup_arrays(X, Y, lambda_=1.0)
    ref = oracle.gblup_fit(X, Y, 1.0)
    assert q == ref["q"]
    assert rel(y_pred, ref["y_pred"]) < TOL_TIGHT
    assert rel(b_hat, ref["b_hat"]) < TOL_CONTRACT


def test_repeated_solves_are_bit_identical():
    """The fused panels and the back substitution exchange data between workgroups of one
    launch through flags; a visibility race would show up as run-to-run differences."""
    n, p = 1000, 800
    X = oracle.synth_genotypes(31, n, p)
    Y = oracle.synth_phenotypes(X, 32, ntraits=2)
    s = gbm.GenotypeSession(X)
    idx = np.arange(n)
    ref = oracle.gblup_fit(X, Y, 0.5)
    first = None
    for _ in range(25):
        _, y_pred, _, _ = s.gblup(idx, Y, lambda_=0.5)
        if first is None:
            first = np.array(y_pred, copy=True)
            assert rel(first, ref["y_pred"]) < TOL_TIGHT
        else:
            assert np.array_equal(y_pred, first)


@pytest.mark.parametrize("g4,g8,g16,group,tail", [(0, -1, -1, 1, 0), (-1, 0, -1, 1, 0), (-1, -1, 0, 1, 0),
                                                 (0, 0, 0, 1, 0), (0, 0, 0, 0, 0), (0, 0, 0, 1, 704)])
def test_cholesky_panel_groups_forced(gbm_env, g4, g8, g16, group, tail):
    """The 4/8/16-panel groups (K = 256/512/1024 trailing updates; the panel phase as one
    chol_group_kernel launch, or with group = 0 as panel / row-update launches of K = 64 j) run
    only on large trailing matrices by default; force them on a small one (the thresholds are
    read at every solve) and compare with the oracle. tail > 0: the last rows (≤ tail) in one dataflow
    launch on the trailing sub-matrix (GBM_CHOL_TAIL_FLOW)."""
    gbm_env.setenv("GBM_CHOL_GROUP_KERNEL", str(group))
    gbm_env.setenv("GBM_CHOL_TAIL_FLOW", str(tail))
    gbm_env.setenv("GBM_CHOL_G4_LIM", str(g4))
    gbm_env.setenv("GBM_CHOL_G8_LIM", str(g8))
    gbm_env.setenv("GBM_CHOL_G16_LIM", str(g16))
    gbm_env.setenv("GBM_UPD64_LIM", "128")
    gbm_env.setenv("GBM_CHOL_FLOW_MAX", "0")  # the launch-per-panel path (not the dataflow one)
    n, p = 1500, 900
    X = oracle.synth_genotypes(77, n, p)
    Y = oracle.synth_phenotypes(X, 78, ntraits=2)
    b_hat, y_pred, mu, q = gbm.gblup_arrays(X, Y, lambda_=0.7)
    ref = oracle.gblup_fit(X, Y, 0.7)
    assert q == ref["q"]
    assert rel(y_pred, ref["y_pred"]) < TOL_TIGHT
    assert rel(mu, ref["mu"]) < TOL_TIGHT
    assert rel(b_hat, ref["b_hat"]) < TOL_CONTRACT


def test_full_size_c2_properties():
    """Config C2 at full size (n = 5 000, p = 50 000, X generated on the device) through
    size-independent properties of the exact solution:
      * mean diag(G) = (n − 1)/n exactly in exact arithmetic (every kept standardised column has
        Σ z² = n − 1, ddof = 1), and G is symmetric;
      * (G + λI) a = y − μ̂1 (the solve's residual), and 1ᵀa = 0 (μ̂ is the GLS estimate);
      * predict's b0 + X b reproduces the GEBVs (src/prediction.jl:228);
    and then the WHOLE fit (GEBVs, μ̂, b̂ over all 50 000 loci, q) against the oracle's own fit of the
    same 5 000 × 50 000 X and y (oracle/oracle.py gblup_fit: numpy/LAPACK, src/gwas.jl:591-597 and
    src/prediction.jl:228 restated), as the bench's parity leg does."""
    import torch

    from gbm import synth
    from gbm.sharded import HipShardStages, LocalComm, assemble_b_hat, sharded_gblup_step

    n, p, lam = 5000, 50000, 1.0
    st = HipShardStages(n, p, nrhs=1, lambda_=lam, device=0)
    st.generate(4242, 0)
    Y = synth.qtl_phenotypes(4242, n, p, 1, device=0)
    st.load_phenotypes(Y)
    st.standardize()
    st.grm_syrk()
    st.grm_reduce()
    q = int(st.q.item())
    npad = st.npad
    Gu = torch.triu(st.G[:npad, :npad]) / q  # the upper tiles hold G·q (scaled in the solve)
    G = (Gu + Gu.T - torch.diag(torch.diagonal(Gu)))[:n, :n]
    assert abs(float(torch.diagonal(G).mean()) - (n - 1) / n) < 1e-12
    G_cpu = G.cpu().numpy()
    assert np.array_equal(G_cpu, G_cpu.T)
    out = sharded_gblup_step(st, LocalComm())
    y_pred, mu = out["y_pred"][:, 0], out["mu"][0]
    a = st.A[0, :n].cpu().numpy()
    resid = G_cpu @ a + lam * a - (Y[:, 0] - mu)
    assert np.abs(resid).max() / np.abs(Y[:, 0] - mu).max() < 1e-10
    assert abs(a.sum()) / np.abs(a).sum() < 1e-10
    b_hat = assemble_b_hat(out["mu"], out["msum"], [out["B"]], p)
    X = st.X[:, :n].T  # device (n, p)
    pred = b_hat[0, 0] + (X @ torch.from_numpy(b_hat[1:, 0]).to(X.device)).cpu().numpy()
    assert rel(pred, y_pred) < TOL_TIGHT
    # the whole C2 fit against the oracle's fit of the same X and Y
    Xh = np.asfortranarray(st.X[:, :n].cpu().numpy().T)  # (n, p) column-major, 2 GB
    del X, st
    ref = oracle.gblup_fit(Xh, Y, lam)
    del Xh
    assert q == ref["q"]
    assert rel(y_pred, ref["y_pred"][:, 0]) < TOL_TIGHT and rel(out["mu"], ref["mu"]) < TOL_TIGHT
    assert rel(b_hat, ref["b_hat"]) < TOL_CONTRACT
    print(f"\nC2 full fit vs oracle: GEBV {rel(y_pred, ref['y_pred'][:, 0]):.2e}, mu {rel(out['mu'], ref['mu']):.2e}, "
          f"b_hat {rel(b_hat, ref['b_hat']):.2e}")


def test_gblup_fit_synthetic_matches_host_fit():
    """gbm_gblup_fit_synthetic (genotypes generated on the device) equals the
    host-buffer fit of the same synthetic X (and the oracle)."""
    n, p = 1030, 2500
    X = oracle.synth_genotypes(4242, n, p)
    Y = oracle.synth_phenotypes(X, 6, ntraits=2)
    b1, y1, mu1, q1 = gbm.gblup_synthetic(4242, n, p, Y, lambda_=1.0)
    b2, y2, mu2, q2 = gbm.gblup_arrays(X, Y, lambda_=1.0)
    assert q1 == q2 and np.array_equal(y1, y2) and np.array_equal(b1, b2) and np.array_equal(mu1, mu2)
    ref = oracle.gblup_fit(X, Y, 1.0)
    assert rel(y1, ref["y_pred"]) < TOL_TIGHT and rel(b1, ref["b_hat"]) < TOL_CONTRACT


def test_concurrent_calls_from_threads():
    """Re-entrancy as cvmultithread! needs (src/cross_validation.jl:159): eight host threads call
    the C ABI at once on one device (own streams, workspaces, helper-stream events per call);
    every result equals the serial one bit for bit."""
    import threading

    cases = []
    for k in range(8):
        n, p = (1030, 1400) if k % 2 == 0 else (333, 1777)
        X = oracle.synth_genotypes(100 + k, n, p)
        Y = oracle.synth_phenotypes(X, 200 + k, ntraits=1 + k % 3)
        cases.append((X, Y))
    serial = [gbm.gblup_arrays(X, Y, lambda_=0.8) for X, Y in cases]
    out = [None] * len(cases)
    errs = []

    def run(k):
        try:
            out[k] = gbm.gblup_arrays(cases[k][0], cases[k][1], lambda_=0.8)
        except Exception as e:  # reported below
            errs.append(repr(e))

    th = [threading.Thread(target=run, args=(k,)) for k in range(len(cases))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for a, b in zip(out, serial):
        assert np.array_equal(a[1], b[1]) and np.array_equal(a[0], b[0])
