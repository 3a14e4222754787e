"""Exact-integer GRM of diploid dosages on the int8 matrix cores (csrc/grm_exact.hip).

G = Σ_j w_j (d_j − t_j/n)(d_j − t_j/n)ᵀ — the GRM of the standardised genotypes of reference
src/gwas.jl:112-126 (before the 1/q), z_ij = (x_ij − m_j)/sd_j with x = d/2 — computed with every locus
weight w_j = 1/var_j as an exact fixed-point integer, int8 digit GEMMs summed exactly in int32, the
centring in int128 and one rounding to fp64. Checked against

* an extended-precision (x87 80-bit) evaluation of the same sum: a few ulps, i.e. EXACT up to the
  final rounding (the fp64 oracle's own SYRK error is far larger),
* the fp64 oracle (oracle/oracle.py: standardise + Z Zᵀ): 1e-13 of max|G|,
* the whole GBLUP fit through the stage path (HipExactShardStages) against oracle.gblup_fit: GEBVs 1e-9,
* edge cases: ragged n and p, monomorphic loci, all-heterozygous loci, rare alleles (wide weight range:
  S = 10 digits), accumulation, a dosage outside {0, 1, 2}.
"""
import ctypes

import numpy as np
import pytest

import gbm
import oracle
from gbm import _lib
from gbm.sharded import HipExactShardStages, LocalComm, assemble_b_hat, sharded_gblup_step

pytestmark = pytest.mark.gpu


def rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(np.abs(np.asarray(b)).max(), 1e-300))


def exact_grm_ld(D):
    """Σ_j w_j (d_j − t_j/n)(d_j − t_j/n)ᵀ in 80-bit long double with w_j computed exactly as the device
    computes it (fp64: n(n − 1)/(n Σd² − t²)); D is (n, p) int."""
    n = D.shape[0]
    Di = D.astype(np.int64)
    t = Di.sum(0)
    s2 = (Di * Di).sum(0)
    num = n * s2 - t * t
    keep = num > 0
    w = np.where(keep, (float(n) * (n - 1.0)) / np.where(keep, num, 1).astype(np.float64), 0.0)
    C = (Di.astype(np.longdouble) - t.astype(np.longdouble) / n) * np.sqrt(w.astype(np.longdouble))
    return C @ C.T, int(keep.sum())


def device_grm(D, accum_G=None):
    import torch
    lib = gbm.load_library()
    n, p = D.shape
    dev = torch.device("cuda", 0)
    Dd = torch.from_numpy(np.ascontiguousarray(D.T.astype(np.int8))).to(dev)  # (p, n) locus rows
    gdim = lib.gbm_dev_gdim(n)
    npad = lib.gbm_dev_npad(n)
    G = torch.zeros((gdim, gdim), dtype=torch.float64, device=dev)
    if accum_G is not None:
        G[:n, :n] = torch.from_numpy(accum_G).to(dev)
    mean = torch.empty(p, dtype=torch.float64, device=dev)
    sd = torch.empty(p, dtype=torch.float64, device=dev)
    keep = torch.empty(p, dtype=torch.int32, device=dev)
    q = torch.zeros(1, dtype=torch.int64, device=dev)
    wsb = lib.gbm_dev_grm_exact_workspace(n, p)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    S = ctypes.c_int32(0)
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    rc = lib.gbm_dev_grm_exact_i8(P(Dd), n, p, n, 2, P(G), gdim, P(mean), P(sd), P(keep), P(q),
                                  1 if accum_G is not None else 0, P(ws), wsb, ctypes.byref(S), stream)
    torch.cuda.synchronize()
    _lib.check(rc, "grm_exact_i8")
    Gh = G.cpu().numpy()[:n, :n]
    Gu = np.triu(Gh)
    return Gu + np.triu(Gu, 1).T, int(q.item()), S.value, mean.cpu().numpy(), sd.cpu().numpy(), keep.cpu().numpy(), npad


def ulps_off(G, Gl):
    """|G − Gl| relative to |Gl| (floored at 1e-3 max|Gl|, where the 80-bit reference's own rounding of
    near-zero entries dominates), in units of u = 2^−53."""
    Gl = np.asarray(Gl)
    den = np.abs(Gl) + 1e-3 * np.abs(Gl).max()
    return float((np.abs(G.astype(np.longdouble) - Gl) / den).max() / 2.0 ** -53)


def random_dosages(seed, n, p, maf_lo=0.05, maf_hi=0.5):
    rng = np.random.default_rng(seed)
    f = rng.uniform(maf_lo, maf_hi, p)
    return rng.binomial(2, f, size=(n, p)).astype(np.int8)


@pytest.mark.parametrize("n,p", [(300, 1000), (257, 3001), (640, 128), (129, 4096)])
def test_exact_grm_matches_extended_precision(n, p):
    D = random_dosages(n * 7 + p, n, p)
    G, q, S, *_ = device_grm(D)
    Gl, ql = exact_grm_ld(D)
    assert q == ql
    assert 8 <= S <= 10
    # one rounding of the int128 bracket, one of the division by n² (+ the ldexp): a few ulps
    assert ulps_off(G, Gl) < 8


def test_exact_grm_matches_fp64_oracle_and_stats():
    n, p = 500, 2000
    D = random_dosages(5, n, p)
    X = D.astype(np.float64) / 2.0
    G, q, S, mean, sd, keep, _ = device_grm(D)
    m, s, kp = oracle.colstats(X)
    Z = oracle.standardize(X, m, s, kp)
    Gref = Z @ Z.T
    assert q == int(kp.sum()) and np.array_equal(keep.astype(bool), kp.astype(bool))
    assert rel(G, Gref) < 1e-13
    assert rel(mean, m) < 1e-14 and rel(sd[kp.astype(bool)], s[kp.astype(bool)]) < 1e-13


def test_exact_grm_edge_loci():
    n, p = 200, 700
    D = random_dosages(9, n, p)
    D[:, 0] = 0          # monomorphic (dropped: keep = 0)
    D[:, 1] = 2          # monomorphic
    D[:, 2] = 1          # all heterozygous: var 0, dropped
    D[:, 3] = 0
    D[5, 3] = 1          # a single carrier: the largest weight (wide range: more digits)
    D[:, 4] = 0
    D[7, 4] = 2
    G, q, S, *_ = device_grm(D)
    Gl, ql = exact_grm_ld(D)
    assert q == ql == p - 3
    assert S >= 9
    assert ulps_off(G, Gl) < 8


def test_exact_grm_wide_weight_range():
    """A single carrier among n = 2000 individuals (var ≈ 1/n) beside balanced loci (var ≈ 1/2): the
    weights span ≈ 2^10, which takes S = 10 digits and stays exact."""
    n, p = 2000, 200
    D = random_dosages(11, n, p, 0.3, 0.5)
    D[:, 0] = 0
    D[17, 0] = 1
    G, q, S, *_ = device_grm(D)
    Gl, _ = exact_grm_ld(D)
    assert S >= 9
    assert ulps_off(G, Gl) < 8


def test_exact_grm_accumulates():
    n, p = 300, 900
    D = random_dosages(3, n, p)
    G0 = np.random.default_rng(1).standard_normal((n, n))
    G0 = G0 + G0.T
    G, *_ = device_grm(D, accum_G=G0)
    Gx, *_ = device_grm(D)
    assert rel(G - G0, Gx) < 1e-14


def test_exact_grm_rejects_bad_dosage():
    D = random_dosages(4, 100, 300)
    D[3, 10] = 3
    with pytest.raises(_lib.ArgumentError):
        device_grm(D)


@pytest.mark.parametrize("n,p,t", [(700, 5000, 2), (1000, 3000, 1)])
def test_exact_stage_gblup_matches_oracle(n, p, t):
    import torch
    seed = 77
    X = oracle.synth_genotypes(seed, n, p)
    Y = oracle.synth_phenotypes(X, seed + 1, ntraits=t)
    st = HipExactShardStages(n, p, nrhs=t, lambda_=1.0, device=0)
    st.generate(seed, 0)
    st.load_phenotypes(Y)
    out = sharded_gblup_step(st, LocalComm())
    torch.cuda.synchronize()
    ref = oracle.gblup_fit(X, Y, 1.0)
    q = int(st.q.item())
    assert q == ref["q"]
    b_hat = assemble_b_hat(out["mu"], out["msum"], [out["B"]], p)
    assert rel(out["y_pred"], ref["y_pred"]) < 1e-9 and rel(out["mu"], ref["mu"]) < 1e-9
    assert rel(b_hat, ref["b_hat"]) < 1e-6
    assert rel(b_hat[0] + X @ b_hat[1:], out["y_pred"]) < 1e-9


def test_exact_full_size_c2_against_fp64_grm():
    """C2 (5 000 x 50 000): the exact GRM against the fp64-MFMA GRM of the same genotypes (rounding of the
    fp64 path only) and mean diag(G)/q = (n − 1)/n."""
    import torch
    from gbm.sharded import HipShardStages
    n, p, seed = 5000, 50000, 4242
    ex = HipExactShardStages(n, p, device=0)
    ex.generate(seed, 0)
    ex.standardize()
    ex.grm_syrk()
    fp = HipShardStages(n, p, device=0)
    fp.generate(seed, 0)
    fp.standardize()
    fp.grm_syrk()
    fp.grm_reduce()
    torch.cuda.synchronize()
    assert int(ex.q.item()) == int(fp.q.item())
    Ge = torch.triu(ex.G[:n, :n])
    Gf = torch.triu(fp.G[:n, :n])
    err = float((Ge - Gf).abs().max() / Gf.abs().max())
    assert err < 1e-12, err
    q = int(ex.q.item())
    assert abs(float(torch.diagonal(ex.G[:n, :n]).mean()) / q - (n - 1) / n) < 1e-12


@pytest.mark.parametrize("devices", [(0,), (0, 0)])
def test_c_abi_exact_synthetic_matches_oracle(gbm_env, devices):
    """gbm_gblup_fit_synthetic with GBM_GRM=exact (the C-ABI entry a Julia ccall binds): one shard, and two
    shards on one device (their exact partial GRMs summed), against the oracle and the fp64 path."""
    n, p, seed = 700, 5000, 77
    X = oracle.synth_genotypes(seed, n, p)
    Y = oracle.synth_phenotypes(X, seed + 1, ntraits=2)
    gbm_env.setenv("GBM_GRM", "exact")
    b, y, mu, q = gbm.gblup_synthetic(seed, n, p, Y, lambda_=1.0, devices=list(devices))
    ref = oracle.gblup_fit(X, Y, 1.0)
    assert q == ref["q"]
    assert rel(y, ref["y_pred"]) < 1e-9 and rel(mu, ref["mu"]) < 1e-9 and rel(b, ref["b_hat"]) < 1e-6
    gbm_env.delenv("GBM_GRM")
    b0, y0, mu0, q0 = gbm.gblup_synthetic(seed, n, p, Y, lambda_=1.0, devices=list(devices))
    assert q0 == q and rel(y, y0) < 1e-11 and rel(b, b0) < 1e-9


def test_c_abi_exact_dosage_matches_oracle(gbm_env):
    n, p = 600, 3000
    D = random_dosages(21, n, p)
    X = D.astype(np.float64) / 2.0
    Y = oracle.synth_phenotypes(X, 5, ntraits=1)
    gbm_env.setenv("GBM_GRM", "exact")
    b, y, mu, q = gbm.gblup_dosage(np.asfortranarray(D), 2, Y)
    ref = oracle.gblup_fit(X, Y, 1.0)
    assert q == ref["q"]
    assert rel(y, ref["y_pred"]) < 1e-9 and rel(b, ref["b_hat"]) < 1e-6


@pytest.mark.parametrize("cus", ["16", "7"])
def test_exact_grm_split_tail(gbm_env, cus):
    """The partial last round of units split into loci ranges (forced on a small shape by pretending a chip
    of 16 or 7 CUs): the ranges' int32 partials summed by the last range to finish, still exact."""
    gbm_env.setenv("GBM_XG_CUS", cus)
    n, p = 700, 1500
    D = random_dosages(31, n, p)
    G, q, S, *_ = device_grm(D)
    Gl, ql = exact_grm_ld(D)
    assert q == ql
    assert ulps_off(G, Gl) < 8


@pytest.mark.parametrize("env", [{"GBM_XG_BM": "64"}, {"GBM_XG_BK": "256"}, {"GBM_XG_ORDER": "1"},
                                 {"GBM_XG_BM": "64", "GBM_XG_CUS": "8"}])
def test_exact_grm_kernel_variants(gbm_env, env):
    """The GEMM's tile (64 x 64, two workgroups per CU), stage (256 loci) and unit-order variants, and the
    split tail of the 64 x 64 grid: the same exact GRM."""
    for k, v in env.items():
        gbm_env.setenv(k, v)
    n, p = 700, 1500
    D = random_dosages(41, n, p)
    G, q, S, *_ = device_grm(D)
    Gl, ql = exact_grm_ld(D)
    assert q == ql
    assert ulps_off(G, Gl) < 8


@pytest.mark.parametrize("source", ["synthetic", "dosage"])
def test_session_exact_training_grm_matches_oracle(gbm_env, source):
    """Sessions of dosage genotypes (synthetic, or int8 with ploidy 2) with GBM_GRM=exact: each training set's
    GRM is the exact-integer one of the gathered training dosages (the CV fold fits of cross_validation.jl and
    the REML path reuse it); fits against the oracle on the same rows, and against the fp64 session."""
    from gbm.session import GenotypeSession
    n, p, seed = 600, 3000, 13
    X = oracle.synth_genotypes(seed, n, p)
    Y = oracle.synth_phenotypes(X, 3, ntraits=2)
    if source == "synthetic":
        make = lambda: GenotypeSession.synthetic(seed, n, p)  # noqa: E731
    else:
        D = np.asfortranarray(np.rint(2.0 * X).astype(np.int8))
        make = lambda: GenotypeSession(dosage_i8=D, ploidy=2)  # noqa: E731
    rng = np.random.default_rng(5)
    idx = np.sort(rng.choice(n, 450, replace=False))
    gbm_env.setenv("GBM_GRM", "exact")
    with make() as s:
        b, y, mu, q = s.gblup(idx, Y[idx])
        va = np.setdiff1d(np.arange(n), idx)
        yv = s.predict(va, b)
    ref = oracle.gblup_fit(X[idx], Y[idx], 1.0)
    assert q == ref["q"]
    assert rel(y, ref["y_pred"]) < 1e-9 and rel(mu, ref["mu"]) < 1e-9 and rel(b, ref["b_hat"]) < 1e-6
    assert rel(yv, oracle.predict_linear(X[va], ref["b_hat"])) < 1e-8
    gbm_env.delenv("GBM_GRM")
    with make() as s:
        b0, y0, mu0, q0 = s.gblup(idx, Y[idx])
    assert q0 == q and rel(y, y0) < 1e-11


@pytest.mark.parametrize("n,p", [(2, 1), (3, 7), (65, 130), (64, 256), (129, 257), (1000, 1)])
def test_exact_grm_tiny_and_ragged_shapes(n, p):
    """The smallest and ragged shapes (a single locus, two individuals, one past the tile edges)."""
    D = random_dosages(n + 13 * p, n, p)
    D[0, :] = 0
    D[-1, :] = 2  # every locus polymorphic
    G, q, S, *_ = device_grm(D)
    Gl, ql = exact_grm_ld(D)
    assert q == ql
    assert ulps_off(G, Gl) < 8


def test_digit_overflow_fails_loudly(gbm_env):
    """Round-4 ADVICE item 2: a locus weight that does not fit its S base-128 digits (fault-injected with
    GBM_XG_TEST_S, one digit fewer than xg_choose's S) makes the exact GRM's status GBM_E_HIP — through the C ABI
    fit (exact and auto alike: it is not a data property, so auto must not hide it), the stage path's download and
    gbm_dev_grm_exact_status — instead of returning a G built from wrong weights."""
    import torch
    n, p = 500, 900
    D = random_dosages(77, n, p)
    D[:, 0] = 0
    D[5, 0] = 1  # a single carrier: the widest weight range (S >= 9)
    _, _, S, *_ = device_grm(D)
    assert S >= 9
    X = D.astype(np.float64) / 2.0
    Y = oracle.synth_phenotypes(X, 3, ntraits=1)
    ref = oracle.gblup_fit(X, Y, 1.0)
    gbm_env.setenv("GBM_XG_TEST_S", str(S - 1))
    for mode in ("exact", "auto"):
        with pytest.raises(gbm.GBMError, match="digits"):
            gbm.gblup_arrays(X, Y, grm=mode)
    st = HipExactShardStages(n, p, nrhs=1, lambda_=1.0, device=0)
    st.D.copy_(torch.from_numpy(np.ascontiguousarray(D.T)).to(st.D.device))
    st.load_phenotypes(Y)
    with pytest.raises(gbm.GBMError, match="digits"):
        sharded_gblup_step(st, LocalComm())
    gbm_env.delenv("GBM_XG_TEST_S")
    out = sharded_gblup_step(st, LocalComm())  # the same shard, the right S: a valid fit
    assert rel(out["y_pred"], ref["y_pred"]) < 1e-9
    b, y, mu, q = gbm.gblup_arrays(X, Y, grm="exact")
    assert rel(y, ref["y_pred"]) < 1e-9
