"""CPU oracle (fp64 numpy/LAPACK) for the GRM + GBLUP hot path — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product: only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it. The product path (``gbm.gblup`` → libgbm.so →
HIP kernels) never calls into ``oracle/`` and fails loudly when the HIP library is missing.

Parity status: **parity unpinned against the reference itself.** The reference is Julia
(GenomicBreedingModels.jl v0.3.0) and the GRM lives in the un-vendored GenomicBreedingCore
(called at reference src/gwas.jl:117-126); ``julia`` is absent from the image and the
reference ships no numeric golden vectors. This file is an
independent restatement of the reference's conventions, pinned by (i) the reference's own
doctest properties (standardised moments within 1e-10, src/gwas.jl:55-62; extractxyetc shape
and content, src/prediction.jl:44-50), (ii) the primal RR-BLUP ≡ dual GBLUP identity and
(iii) a second, independent C restatement (oracle/gbm_oracle.c). See DESIGN.md "Oracle".

Every function cites the reference lines it restates.
"""
from __future__ import annotations

import numpy as np

EPS64 = np.finfo(np.float64).eps

# ----------------------------------------------------------------------------------------
# Synthetic genotypes: counter-based hash. Identical integer arithmetic to
# oracle/gbm_oracle.c and the HIP generator kernel, so X is bit-identical everywhere.
# ----------------------------------------------------------------------------------------
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
_GOLD = np.uint64(0x9E3779B97F4A7C15)
_C1 = np.uint64(0xBF58476D1CE4E5B9)
_C2 = np.uint64(0x94D049BB133111EB)
_KJ = np.uint64(0xD1B54A32D192ED03)
_KI = np.uint64(0x8CB92BA72F3D8DD7)
_F_LO = np.uint64(214748364)     # floor(0.05 * 2^32)
_F_SPAN = np.uint64(1932735283)  # floor(0.45 * 2^32)


def _mix64(z):
    """splitmix64 finalizer on uint64 arrays (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = (z + _GOLD).astype(np.uint64)
        z = ((z ^ (z >> np.uint64(30))) * _C1).astype(np.uint64)
        z = ((z ^ (z >> np.uint64(27))) * _C2).astype(np.uint64)
        return z ^ (z >> np.uint64(31))


def synth_locus_threshold(seed: int, j):
    """32-bit threshold t_j with f_j = t_j / 2^32 ∈ [0.05, 0.5)."""
    j = np.asarray(j, dtype=np.uint64)
    with np.errstate(over="ignore"):
        base = _mix64(np.uint64(seed) * _KJ + j)
    return _F_LO + (((base >> np.uint64(32)) * _F_SPAN) >> np.uint64(32))


def synth_genotypes(seed: int, n: int, p: int, j0: int = 0) -> np.ndarray:
    """X (n x p, Fortran order like Julia) with X[i, j] = dosage/2 of locus j0 + j."""
    j = np.arange(j0, j0 + p, dtype=np.uint64)
    i = np.arange(n, dtype=np.uint64)
    thr = synth_locus_threshold(seed, j)  # (p,)
    with np.errstate(over="ignore"):
        base = _mix64(np.uint64(seed) * _KJ + j)  # (p,)
        h = _mix64(base[None, :] ^ (i[:, None] * _KI))  # (n, p)
    u1 = h & np.uint64(0xFFFFFFFF)
    u2 = h >> np.uint64(32)
    d = (u1 < thr[None, :]).astype(np.int8) + (u2 < thr[None, :]).astype(np.int8)
    return np.asfortranarray(d.astype(np.float64) * 0.5)


def synth_phenotypes(X: np.ndarray, seed: int, ntraits: int = 1, qtl_frac: float = 0.01,
                     h2: float = 0.5) -> np.ndarray:
    """y = Xβ + e with 1% QTL effects N(0,1) and e ~ N(0, var(g)(1-h²)/h²)."""
    n, p = X.shape
    rng = np.random.default_rng(seed)
    Y = np.empty((n, ntraits))
    for t in range(ntraits):
        nq = max(1, int(round(qtl_frac * p)))
        idx = rng.choice(p, size=nq, replace=False)
        beta = rng.standard_normal(nq)
        g = X[:, idx] @ beta
        vg = g.var(ddof=1) if n > 1 else 1.0
        ve = vg * (1.0 - h2) / h2 if vg > 0 else 1.0
        Y[:, t] = g + rng.standard_normal(n) * np.sqrt(ve)
    return Y


# ----------------------------------------------------------------------------------------
# The hot path restated.
# ----------------------------------------------------------------------------------------

def colstats(X: np.ndarray):
    """mean, std (ddof=1, Julia ``std``) and the keep mask of reference src/gwas.jl:112-113:
    ``v = std(G, dims=1)``; keep ``v .> eps(Float64)`` and finite."""
    n = X.shape[0]
    m = X.mean(axis=0)
    if n > 1:
        s = np.sqrt(((X - m) ** 2).sum(axis=0) / (n - 1))
    else:
        s = np.full(X.shape[1], np.nan)
    keep = (s > EPS64) & np.isfinite(s)
    return m, s, keep


def standardize(X: np.ndarray, m: np.ndarray, s: np.ndarray, keep: np.ndarray) -> np.ndarray:
    """Z = (X − m)/s over kept columns (reference src/gwas.jl:114,129)."""
    return (X[:, keep] - m[keep]) / s[keep]


def grm(X: np.ndarray):
    """G = Z Zᵀ / q (north_star; replaces Core's grmsimple called at src/gwas.jl:124)."""
    m, s, keep = colstats(X)
    Z = standardize(X, m, s, keep)
    q = Z.shape[1]
    if q == 0:
        raise ValueError("no polymorphic locus")
    return (Z @ Z.T) / q, q


def grm_ploidy_aware(X: np.ndarray, ploidy: int):
    """Ploidy-aware GRM for GenomicBreedingCore.grmploidyaware, called at src/gwas.jl:117-121 —
    un-vendored, so this is a restatement of VanRaden (2008) generalised to ploidy k (parity
    unpinned): dosages kX, f = column means, G = (kX − k1fᵀ)(kX − k1fᵀ)ᵀ / (k Σ f(1 − f)).
    Written in dosage units, independently of the device's centred-frequency form."""
    D = ploidy * X
    f = X.mean(axis=0)
    P = ploidy * f
    den = float((f * (1.0 - f)).sum())
    if not den > 0.0:
        raise ValueError("no polymorphic locus")
    return ((D - P) @ (D - P).T) / (ploidy * den), den


def gblup_fit(X: np.ndarray, Y: np.ndarray, lam: float = 1.0) -> dict:
    """GBLUP on V = G + λI (reference src/gwas.jl:462-471 with σ²_u = 1, σ²_e = λ).

    μ̂ = 1ᵀV⁻¹y / 1ᵀV⁻¹1 (GLS, src/gwas.jl:596 with X = 1), a = V⁻¹(y − 1μ̂),
    GEBV = μ̂ + G a, marker effects b_j = (Zᵀa)_j/(q s_j), b0 = μ̂ − Σ m_j b_j so that
    ``b_hat[1] .+ X*b_hat[2:end]`` (src/prediction.jl:228) reproduces the GEBVs.
    Y may be (n,) or (n, t). Returns a dict of fp64 arrays (trait along the last axis).
    """
    import scipy.linalg as sla

    X = np.asarray(X, dtype=np.float64)
    Y = np.asarray(Y, dtype=np.float64)
    if Y.ndim == 1:
        Y = Y[:, None]
    n, p = X.shape
    m, s, keep = colstats(X)
    Z = standardize(X, m, s, keep)
    q = Z.shape[1]
    if q == 0:
        raise ValueError("no polymorphic locus")
    G = (Z @ Z.T) / q
    V = G + lam * np.eye(n)
    c = sla.cho_factor(V, lower=True)
    ones = np.ones(n)
    vi1 = sla.cho_solve(c, ones)
    viy = sla.cho_solve(c, Y)
    mu = (ones @ viy) / (ones @ vi1)
    R = Y - mu[None, :]
    A = sla.cho_solve(c, R)
    U = R - lam * A  # = G a  (since (G + λI) a = R)
    gebv = mu[None, :] + U
    beta_std = (Z.T @ A) / q  # (q, t)
    B = np.zeros((p, Y.shape[1]))
    B[keep, :] = beta_std / s[keep][:, None]
    b0 = mu - m @ B
    b_hat = np.vstack([b0[None, :], B])
    return dict(b_hat=b_hat, y_pred=gebv, mu=mu, q=q, a=A, G=G, mean=m, sd=s, keep=keep)


def rrblup_primal(X: np.ndarray, y: np.ndarray, lam: float, mu: float):
    """Primal ridge form (ZᵀZ + qλI)β = Zᵀ(y − μ̂) — must equal the dual GBLUP β̃ (known-answer
    identity used to pin the oracle)."""
    m, s, keep = colstats(X)
    Z = standardize(X, m, s, keep)
    q = Z.shape[1]
    lhs = Z.T @ Z + q * lam * np.eye(q)
    return np.linalg.solve(lhs, Z.T @ (y - mu))


def predict_linear(X: np.ndarray, b_hat: np.ndarray) -> np.ndarray:
    """``b_hat[1] .+ X*b_hat[2:end]`` (reference src/prediction.jl:228)."""
    return b_hat[0] + X @ b_hat[1:]


# ----------------------------------------------------------------------------------------
# metrics (reference src/metrics.jl:23-128; Distances.jl semantics restated)
# ----------------------------------------------------------------------------------------

def metrics(y_true: np.ndarray, y_pred: np.ndarray) -> dict:
    y_true = np.asarray(y_true, dtype=np.float64)
    y_pred = np.asarray(y_pred, dtype=np.float64)

    def var(v):
        return v.var(ddof=1) if v.size > 1 else np.nan

    low = (var(y_true) < 1e-10) or (var(y_pred) < 1e-10)
    d = y_true - y_pred
    if low:
        cor = 0.0
        r2 = 0.0
        h2 = 0.0
    else:
        a = y_true - y_true.mean()
        b = y_pred - y_pred.mean()
        cor = float(1.0 - (1.0 - (a @ b) / np.sqrt((a @ a) * (b @ b))))
        r2 = float(1.0 - var(d) / var(y_true))
        s2a = var(y_pred)
        s2e = var(d)
        h2 = s2a / (s2a + s2e) if (s2a + s2e) >= 1e-20 else 0.0
        h2 = float(min(max(h2, 0.0), 1.0))
    msd = float(np.mean(d * d))
    rmsd = float(np.sqrt(msd))
    return {
        "cor": cor,
        "mad": float(np.mean(np.abs(d))),
        "msd": msd,
        "rmsd": rmsd,
        "nrmsd": float(rmsd / (y_true.max() - y_true.min())),
        "euc": float(np.sqrt(np.sum(d * d))),
        "jac": float(1.0 - np.sum(np.minimum(y_true, y_pred)) / np.sum(np.maximum(y_true, y_pred))),
        "tvar": float(0.5 * np.sum(np.abs(d))),
        "h²": h2,
        "r²": r2,
    }


# ----------------------------------------------------------------------------------------
# REML
# ----------------------------------------------------------------------------------------
def loglikreml(theta, y: np.ndarray, Xf: np.ndarray, GRM: np.ndarray) -> float:
    """Reference ``loglikreml`` (src/gwas.jl:450-483) restated line for line: V = σ²_u GRM + σ²_e I,
    V⁻¹ by pinv, P = V⁻¹ − V⁻¹X(XᵀV⁻¹X)⁻¹XᵀV⁻¹, objective 0.5 log det V + yᵀPy + log det(XᵀV⁻¹X)."""
    s2e, s2u = float(theta[0]), float(theta[1])
    V = s2u * GRM + s2e * np.eye(GRM.shape[0])
    Vi = np.linalg.pinv(V)
    XtViX = Xf.T @ Vi @ Xf
    P = Vi - Vi @ Xf @ np.linalg.inv(XtViX) @ Xf.T @ Vi
    sign, logdet = np.linalg.slogdet(V)
    return 0.5 * logdet + float(y @ (P @ y)) + float(np.log(np.linalg.det(XtViX)))


def reml_reference(y: np.ndarray, GRM: np.ndarray) -> dict:
    """What the reference's REML does for an intercept-only model: y standardised as in gwasprep
    (src/gwas.jl:127-128), L-BFGS over θ = [σ²_e, σ²_u] ∈ [eps, 1]² from [0.5, 0.5] with
    g_tol 1e-4 (src/gwas.jl:577-590; Optimization.jl's LBFGS there, scipy's L-BFGS-B here)."""
    from scipy.optimize import minimize

    ys = (y - y.mean()) / y.std(ddof=1)
    Xf = np.ones((y.size, 1))
    res = minimize(lambda th: loglikreml(th, ys, Xf, GRM), x0=[0.5, 0.5], method="L-BFGS-B",
                   bounds=[(EPS64, 1.0), (EPS64, 1.0)], options={"gtol": 1e-10, "ftol": 1e-15, "maxiter": 500})
    return {"sigma2_e": float(res.x[0]), "sigma2_u": float(res.x[1]), "lambda": float(res.x[0] / res.x[1]),
            "objective": float(res.fun), "y_std": ys}


def lmm_gls_loglik(y: np.ndarray, X: np.ndarray, V: np.ndarray, reml: bool) -> dict:
    """Textbook linear-mixed-model quantities at given variance components, V = cov(y) (dense
    Cholesky): GLS β̂ = (XᵀV⁻¹X)⁻¹XᵀV⁻¹y, vcov(β̂) = (XᵀV⁻¹X)⁻¹ and the ML or REML (Harville)
    log-likelihood −½[(n − p_ml) log 2π + log det V (+ log det XᵀV⁻¹X) + (y − Xβ̂)ᵀV⁻¹(y − Xβ̂)].
    The same GLS/logdet machinery as the reference's V/GLS equations (src/gwas.jl:462-472,591-597)
    and loglikreml (:450-483), in the form R lme4 reports: it pins this oracle (and the device
    solve's terms) against lme4 known answers (tests/golden/lmer_r.npz)."""
    import scipy.linalg as sla

    n, pf = X.shape
    c = sla.cho_factor(V, lower=True)
    ViX = sla.cho_solve(c, X)
    Viy = sla.cho_solve(c, y)
    M = X.T @ ViX
    beta = np.linalg.solve(M, X.T @ Viy)
    r = float(y @ Viy - beta @ (X.T @ Viy))
    logdet = 2.0 * float(np.log(np.diag(c[0])).sum())
    if reml:
        ll = -0.5 * ((n - pf) * np.log(2 * np.pi) + logdet + np.linalg.slogdet(M)[1] + r)
    else:
        ll = -0.5 * (n * np.log(2 * np.pi) + logdet + r)
    return {"beta": beta, "vcov": np.linalg.inv(M), "loglike": float(ll), "logdet": logdet}


# ----------------------------------------------------------------------------------------
# Ridge path: GLMNet alpha = 0, standardize = false, intercept
# (reference ridge, src/linear.jl:193-203). glmnet is un-vendored; restated from its published
# objective (1/2n)‖y − a0 − Xb‖² + (λ/2)‖b‖² and pinned by R-glmnet known answers
# (tests/golden/glmnet_ridge_r.npz).
# ----------------------------------------------------------------------------------------
def ridge_exact(X: np.ndarray, y: np.ndarray, lam: float):
    """Exact glmnet ridge minimiser: (X_cᵀX_c + (nλ/σ_y)I) b = X_cᵀ(y − ȳ), a0 = ȳ − x̄ᵀb.

    glmnet's gaussian elnet (libglmnet, called by GLMNet.jl in the reference ``ridge``,
    src/linear.jl:193-203) scales y by its population sd σ_y = sqrt(mean((y − ȳ)²)) and divides the
    user λ by the same σ_y (vlam = ulam/ys) before its coordinate descent, then rescales b by σ_y:
    on the original scale the penalty is λ/σ_y."""
    n, p = X.shape
    xm, ym = X.mean(axis=0), y.mean()
    ys = float(np.sqrt(np.mean((y - ym) ** 2)))
    Xc = X - xm
    pen = n * lam / ys
    if p <= n:
        b = np.linalg.solve(Xc.T @ Xc + pen * np.eye(p), Xc.T @ (y - ym))
    else:
        b = Xc.T @ np.linalg.solve(Xc @ Xc.T + pen * np.eye(n), y - ym)
    return ym - xm @ b, b


def ridge_lambda_max(X: np.ndarray, y: np.ndarray) -> float:
    """glmnet's first λ for alpha = 0 (alpha floored at 1e-3 in the λ_max formula)."""
    Xc = X - X.mean(axis=0)
    return float(np.abs(Xc.T @ (y - y.mean())).max() / X.shape[0] / 1e-3)


def ridge_path_cv(X, y, folds, nlambda=100, lambda_min_ratio=0.01):
    """glmnetcv's λ path, exact path solutions and CV mean squared error for given fold labels."""
    lam = ridge_lambda_max(X, y) * lambda_min_ratio ** (np.arange(nlambda) / (nlambda - 1))
    a0 = np.zeros(nlambda)
    betas = np.zeros((X.shape[1], nlambda))
    for k, l in enumerate(lam):
        a0[k], betas[:, k] = ridge_exact(X, y, l)
    nf = int(folds.max())
    loss = np.zeros((nlambda, nf))
    for f in range(1, nf + 1):
        tr, ho = folds != f, folds == f
        for k, l in enumerate(lam):
            a, b = ridge_exact(X[tr], y[tr], l)
            loss[k, f - 1] = np.mean((a + X[ho] @ b - y[ho]) ** 2)
    return {"lambda": lam, "a0": a0, "betas": betas, "meanloss": loss.mean(axis=1)}


# ----------------------------------------------------------------------------------------
# Bayesian ridge regression, BGLR model "BRR" (SURVEY.md §8f row 3). BGLR (R, C sampler) is
# un-vendored and absent: restated from its published algorithm (setLT.BRR priors, sample_beta
# single-site updates, scaled-inverse-χ² variance draws, running means every `thin` after
# burn-in), driven by the same counter-based random numbers as the device sampler
# (genomicbreedingmodels.jl_amd/csrc/gibbs.hip) so both follow one sample path.
# ----------------------------------------------------------------------------------------
_U64 = (1 << 64) - 1


def _mix_int(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & _U64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _U64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _U64
    return z ^ (z >> 31)


def brr_u01(seed: int, a: int, b: int) -> float:
    h = _mix_int(_mix_int(seed ^ ((a * 0xD1B54A32D192ED03) & _U64)) ^ ((b * 0x8CB92BA72F3D8DD7) & _U64))
    return ((h >> 11) + 0.5) * 2.0 ** -53


def brr_normal(seed: int, a: int, b: int) -> float:
    import math
    u1, u2 = brr_u01(seed, a, 2 * b), brr_u01(seed, a, 2 * b + 1)
    return math.sqrt(-2.0 * math.log(u1)) * math.cos(6.283185307179586 * u2)


def brr_chisq(seed: int, a: int, df: float) -> float:
    """χ²(df) = 2 Gamma(df/2), Marsaglia-Tsang; attempt t: normal (a, 2t), uniform (a, 4t+2)."""
    import math
    d = 0.5 * df - 1.0 / 3.0
    c = 1.0 / math.sqrt(9.0 * d)
    for t in range(1000):
        x = brr_normal(seed, a, 2 * t)
        v = 1.0 + c * x
        if v <= 0.0:
            continue
        v = v * v * v
        u = brr_u01(seed, a, 4 * t + 2)
        if math.log(u) < 0.5 * x * x + d - d * v + d * math.log(v):
            return 2.0 * d * v
    return df


def brr_gibbs(X: np.ndarray, y: np.ndarray, n_iter: int, n_burnin: int, thin: int = 5, r2: float = 0.5,
              df0: float = 5.0, seed: int = 42) -> dict:
    """BGLR's BRR Gibbs sampler (single site, un-blocked) — the oracle for gbm_brr_fit."""
    n, p = X.shape
    X = np.asarray(X, dtype=np.float64)
    x2 = (X * X).sum(axis=0)
    msx = x2.sum() / n - (X.mean(axis=0) ** 2).sum()
    vy = y.var(ddof=1)
    S0e, S0b = vy * (1 - r2) * (df0 + 2), vy * r2 / msx * (df0 + 2)
    varE, varB = S0e / (df0 + 2), S0b / (df0 + 2)
    mu = y.mean()
    e = y - mu
    b = np.zeros(p)
    bbar = np.zeros(p)
    mubar = varEbar = varBbar = 0.0
    nsum = 0
    for it in range(n_iter):
        a = 4 * it
        s = (e + mu).sum()
        mu_new = s / n + np.sqrt(varE / n) * brr_normal(seed, a, 0xFFFFFFFF)
        e = (e + mu) - mu_new
        mu = mu_new
        for j in range(p):
            xj = X[:, j]
            rhs = (xj @ e) / varE + x2[j] * b[j] / varE
            c = x2[j] / varE + 1.0 / varB
            bn = rhs / c + np.sqrt(1.0 / c) * brr_normal(seed, a, j)
            e += (b[j] - bn) * xj
            b[j] = bn
        varB = ((b * b).sum() + S0b) / brr_chisq(seed, a + 1, df0 + p)
        varE = ((e * e).sum() + S0e) / brr_chisq(seed, a + 2, df0 + n)
        i = it + 1
        if i % thin == 0 and i > n_burnin:
            nsum += 1
            k = float(nsum)
            bbar = bbar * ((k - 1) / k) + b / k
            mubar = mubar * ((k - 1) / k) + mu / k
            varEbar = varEbar * ((k - 1) / k) + varE / k
            varBbar = varBbar * ((k - 1) / k) + varB / k
    b_hat = np.concatenate([[mubar], bbar])
    return {"b_hat": b_hat, "y_pred": mubar + X @ bbar, "varE": varEbar, "varB": varBbar, "b_last": b, "mu_last": mu}
