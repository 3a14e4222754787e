"""Extract R lme4 known answers for linear mixed models from the statsmodels test suite shipped in
this image (statsmodels/regression/tests: results/lme00.csv .. lme11.csv + lme_r_results.py, written
by R's lme4 via the suite's generate_lme.py / lme_results.R; results/dietox.csv with the
lmer(Weight ~ Time + (1 | Pig)) answers quoted in test_lme.py::test_dietox; BSD-licensed test data)
into tests/golden/lmer_r.npz. Used by tests/test_lmer_known_answers.py.

Each case k stores, under keys "k<k>_<name>": y (n), X (n x pf fixed-effect design; a column of
ones where the model has an intercept), Z (n x (ngroups * pr) random-effect design, block per group),
pr, cov_re (pr x pr, R's estimate), scale (R's σ²), coef (R's fixed effects), vcov (R's
(XᵀV⁻¹X)⁻¹ at those estimates), loglike (R's log-likelihood), reml (1 = REML, 0 = ML), intercept
(1 if X's first column is the intercept). The model: y = Xβ + Zu + e, u ~ N(0, I_groups ⊗ cov_re),
e ~ N(0, scale I), so V = Z (I ⊗ cov_re) Zᵀ + scale I."""
import importlib.util
import os

import numpy as np

SRC = "/opt/conda/lib/python3.9/site-packages/statsmodels/regression/tests/results"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lmer_r.npz")

spec = importlib.util.spec_from_file_location("lme_r_results", os.path.join(SRC, "lme_r_results.py"))
R = importlib.util.module_from_spec(spec)
spec.loader.exec_module(R)


def design(groups, zcols):
    """Block random-effect design: row i's pr covariates in the columns of its group."""
    labels, gidx = np.unique(groups, return_inverse=True)
    n, pr = zcols.shape
    Z = np.zeros((n, labels.size * pr))
    for c in range(pr):
        Z[np.arange(n), gidx * pr + c] = zcols[:, c]
    return Z


out = {}
k = 0
for ds in range(12):
    d = np.genfromtxt(os.path.join(SRC, f"lme{ds:02d}.csv"), delimiter=",", names=True)
    names = d.dtype.names
    fe = [c for c in names if c.startswith("exog_fe")]
    re = [c for c in names if c.startswith("exog_re")]
    y = np.asarray(d["endog"], dtype=np.float64)
    X = np.column_stack([d[c] for c in fe]).astype(np.float64)
    Z = design(d["groups"], np.column_stack([d[c] for c in re]).astype(np.float64))
    for meth in ("ml", "reml"):
        b = f"_{meth}_drf_{ds}"
        out.update({f"k{k}_y": y, f"k{k}_X": X, f"k{k}_Z": Z, f"k{k}_pr": np.int64(len(re)),
                    f"k{k}_cov_re": np.atleast_2d(getattr(R, "cov_re" + b)).astype(np.float64),
                    f"k{k}_scale": np.float64(getattr(R, "scale" + b)[0]),
                    f"k{k}_coef": np.asarray(getattr(R, "coef" + b), dtype=np.float64),
                    f"k{k}_vcov": np.atleast_2d(getattr(R, "vcov" + b)).astype(np.float64),
                    f"k{k}_loglike": np.float64(getattr(R, "loglike" + b)[0]),
                    f"k{k}_reml": np.int64(meth == "reml"), f"k{k}_intercept": np.int64(0),
                    f"k{k}_name": np.array(f"lme{ds:02d} {meth}")})
        k += 1

# dietox (geepack): lmer(Weight ~ Time + (1 | Pig), data = dietox), REML and REML = FALSE; the
# values are those quoted in statsmodels' test_lme.py::test_dietox (fixef, sqrt(diag(vcov)),
# sigma², the Pig variance, logLik)
rows = []
with open(os.path.join(SRC, "dietox.csv")) as f:
    head = [h.strip('"') for h in f.readline().strip().split(",")]
    for line in f:
        v = line.strip().split(",")[1:]  # the leading field is R's row name (no header entry)
        rows.append((float(v[head.index("Weight")]), float(v[head.index("Time")]), float(v[head.index("Pig")])))
a = np.array(rows)
y, t, pig = a[:, 0], a[:, 1], a[:, 2]
X = np.column_stack([np.ones_like(t), t])
Z = design(pig, np.ones((y.size, 1)))
for reml, fe, bse, scale, cov_re, ll in [
        (1, (15.723523, 6.942505), (0.78805374, 0.03338727), 11.36692, 40.39395, -2404.775),
        (0, (15.723517, 6.942506), (0.7829397, 0.0333661), 11.35251, 39.82097, -2402.932)]:
    out.update({f"k{k}_y": y, f"k{k}_X": X, f"k{k}_Z": Z, f"k{k}_pr": np.int64(1),
                f"k{k}_cov_re": np.array([[cov_re]]), f"k{k}_scale": np.float64(scale),
                f"k{k}_coef": np.array(fe), f"k{k}_vcov": np.diag(np.array(bse) ** 2),
                f"k{k}_bse_only": np.int64(1), f"k{k}_loglike": np.float64(ll), f"k{k}_reml": np.int64(reml),
                f"k{k}_intercept": np.int64(1), f"k{k}_name": np.array("dietox " + ("reml" if reml else "ml"))})
    k += 1
out["ncases"] = np.int64(k)
np.savez_compressed(OUT, **out)
print(OUT, k, "cases")
