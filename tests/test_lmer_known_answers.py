"""External known answers for the mixed-model solve: R lme4 fits from the statsmodels test suite
(tests/golden/lmer_r.npz, made by tests/golden/make_lmer_fixture.py; 12 simulated random-intercept
and random-slope data sets, ML and REML, plus lmer(Weight ~ Time + (1 | Pig)) on dietox).

The GBLUP core's V/GLS machinery (reference src/gwas.jl:462-472,591-597 and the terms of
loglikreml, :450-483) has no numeric golden vector in the reference (parity unpinned);
these R answers pin it from outside. At R's variance-component estimates, with
V = Z (I ⊗ cov_re) Zᵀ + scale I: the GLS fixed effects, their covariance (XᵀV⁻¹X)⁻¹ and the ML /
REML log-likelihood must equal lme4's to the digits R printed.
  * CPU: the oracle's dense restatement (oracle.lmm_gls_loglik);
  * GPU: the device solve — gbm_dev_gblup_solve's bordered Cholesky of G/q + λI with G = V/scale − I,
    q = 1, λ = 1 — and gbm_dev_gblup_terms (log det, 1ᵀV⁻¹1, 1ᵀV⁻¹r, rᵀV⁻¹r per right-hand side);
    cross products xᵀV⁻¹y by polarisation from the right-hand sides x, y, x + y; and a textbook REML
    optimisation driven by those device terms recovers lme4's variance components."""
import os

import numpy as np
import pytest

import oracle

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lmer_r.npz")


def cases():
    d = np.load(FIX)
    out = []
    for k in range(int(d["ncases"])):
        c = {name[len(f"k{k}_"):]: d[name] for name in d.files if name.startswith(f"k{k}_")}
        c["name"] = str(c["name"])
        out.append(c)
    return out


CASES = cases()


def V_of(c, cov_re=None, scale=None):
    cov_re = c["cov_re"] if cov_re is None else cov_re
    scale = float(c["scale"]) if scale is None else scale
    Z, pr = c["Z"], int(c["pr"])
    ng = Z.shape[1] // pr
    return Z @ np.kron(np.eye(ng), cov_re) @ Z.T + scale * np.eye(Z.shape[0])


def check(c, beta, vcov, ll):
    # R printed 7 significant digits
    assert np.allclose(beta, c["coef"], rtol=2e-6, atol=1e-7), (c["name"], beta, c["coef"])
    if int(c.get("bse_only", 0)):
        assert np.allclose(np.sqrt(np.diag(vcov)), np.sqrt(np.diag(c["vcov"])), rtol=2e-6), c["name"]
    else:
        assert np.allclose(vcov, c["vcov"], rtol=2e-6, atol=1e-9), (c["name"], vcov, c["vcov"])
    assert abs(ll - float(c["loglike"])) < 6e-4 + 1e-7 * abs(float(c["loglike"])), (c["name"], ll, c["loglike"])


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_lme4(c):
    r = oracle.lmm_gls_loglik(c["y"], c["X"], V_of(c), bool(c["reml"]))
    check(c, r["beta"], r["vcov"], r["loglike"])


# ---- the device solve -------------------------------------------------------------------------

def device_terms(c, cov_re=None, scale=None, stages_cache={}):
    """gbm_dev_gblup_solve + gbm_dev_gblup_terms on G = V/scale − I (q = 1, λ = 1), right-hand
    sides [x_j (non-intercept columns)..., y, x_a + x_b (a < b), x_j + y]. Returns the GLS
    ingredients on V's scale: logdet V, XᵀV⁻¹X, XᵀV⁻¹y, yᵀV⁻¹y."""
    import ctypes

    import torch

    from gbm import _lib
    from gbm.sharded import HipShardStages
    scale = float(c["scale"]) if scale is None else scale
    y, X = c["y"], c["X"]
    n = y.size
    icpt = bool(int(c["intercept"]))
    xs = X[:, 1:] if icpt else X
    m = xs.shape[1]
    rhs = [xs[:, a] for a in range(m)] + [y]
    pairs = [(a, b) for a in range(m + 1) for b in range(a + 1, m + 1)]
    rhs += [rhs[a] + rhs[b] for a, b in pairs]
    R = len(rhs)
    key = (n, R)
    if key not in stages_cache:
        stages_cache[key] = HipShardStages(n, 1, nrhs=R, lambda_=1.0, device=0)
    st = stages_cache[key]
    Gp = V_of(c, cov_re, scale) / scale - np.eye(n)
    st.G.zero_()
    st.G[:n, :n].copy_(torch.from_numpy(Gp))
    st.q.fill_(1)
    st.load_phenotypes(np.column_stack(rhs))
    st.solve()
    terms = torch.zeros(2 + 2 * R, dtype=torch.float64, device=st.dev)
    _lib.check(st.lib.gbm_dev_gblup_terms(st._p(st.G), st.gdim, n, R, st._p(st.ws_solve), ctypes.c_void_p(terms.data_ptr()),
                                          st._stream()), "terms")
    torch.cuda.synchronize()
    assert int(st.info.item()) == 0
    t = terms.cpu().numpy()
    quad = np.empty((m + 1, m + 1))  # [x..., y] Gram in V'⁻¹ (V' = V/scale)
    for a in range(m + 1):
        quad[a, a] = t[3 + 2 * a]
    for k, (a, b) in enumerate(pairs):
        quad[a, b] = quad[b, a] = 0.5 * (t[3 + 2 * (m + 1 + k)] - quad[a, a] - quad[b, b])
    one = np.array([t[2 + 2 * a] for a in range(m + 1)])  # 1ᵀV'⁻¹[x..., y]
    if icpt:
        full = np.empty((m + 2, m + 2))
        full[0, 0] = t[1]
        full[0, 1:] = full[1:, 0] = one
        full[1:, 1:] = quad
    else:
        full = quad
    p1 = full.shape[0] - 1  # fixed-effect columns; the last index is y
    return {"logdet": n * np.log(scale) + t[0], "M": full[:p1, :p1] / scale, "b": full[:p1, p1] / scale,
            "yy": full[p1, p1] / scale, "n": n, "pf": p1}


def loglik_of(d, reml):
    beta = np.linalg.solve(d["M"], d["b"])
    r = d["yy"] - beta @ d["b"]
    if reml:
        ll = -0.5 * ((d["n"] - d["pf"]) * np.log(2 * np.pi) + d["logdet"] + np.linalg.slogdet(d["M"])[1] + r)
    else:
        ll = -0.5 * (d["n"] * np.log(2 * np.pi) + d["logdet"] + r)
    return beta, np.linalg.inv(d["M"]), float(ll)


@pytest.mark.gpu
@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_device_solve_matches_lme4(c):
    beta, vcov, ll = loglik_of(device_terms(c), bool(c["reml"]))
    check(c, beta, vcov, ll)
    ref = oracle.lmm_gls_loglik(c["y"], c["X"], V_of(c), bool(c["reml"]))
    assert np.allclose(beta, ref["beta"], rtol=1e-9, atol=1e-12) and abs(ll - ref["loglike"]) < 1e-8 * abs(ll)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["lme00 reml", "lme03 ml", "lme05 reml", "dietox reml", "dietox ml"])
def test_device_variance_components_match_lme4(name):
    """Random-intercept models: maximise the ML / REML log-likelihood over (cov_re, scale), every
    evaluation through the device solve's terms; the optimum is lme4's (to its printed digits and
    the optimiser's tolerance)."""
    from scipy.optimize import minimize
    c = next(c for c in CASES if c["name"] == name)
    reml = bool(c["reml"])

    def f(th):
        cr, sc = np.exp(th)
        return -loglik_of(device_terms(c, np.array([[cr]]), sc), reml)[2]

    x0 = np.log([float(c["cov_re"][0, 0]) * 1.7 + 1e-3, float(c["scale"]) * 0.6])
    res = minimize(f, x0, method="Nelder-Mead", options={"xatol": 1e-7, "fatol": 1e-10, "maxiter": 2000})
    cr, sc = np.exp(res.x)
    assert abs(cr - float(c["cov_re"][0, 0])) < 2e-4 * float(c["cov_re"][0, 0]) + 1e-6, (cr, c["cov_re"])
    assert abs(sc - float(c["scale"])) < 2e-4 * float(c["scale"]), (sc, c["scale"])
    assert abs(-res.fun - float(c["loglike"])) < 6e-4 + 1e-7 * abs(float(c["loglike"]))
