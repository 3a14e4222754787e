"""Extract R-glmnet known answers for ridge (alpha = 0) from the statsmodels test suite shipped in
this image (statsmodels/regression/tests/results: lasso_data.csv + glmnet_r_results.py, written by
R's glmnet; BSD-licensed test data) into tests/golden/glmnet_ridge_r.npz. Each case: the first n
rows and p columns of the data, y and X centred and scaled (ddof=1) as the statsmodels harness does
(test_regression.py:1063-1066), λ, and glmnet's coefficients. Used by tests/test_ridge.py."""
import importlib.util
import os

import numpy as np

SRC = "/opt/conda/lib/python3.9/site-packages/statsmodels/regression/tests/results"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "glmnet_ridge_r.npz")

data = np.loadtxt(os.path.join(SRC, "lasso_data.csv"), delimiter=",")
spec = importlib.util.spec_from_file_location("glmnet_r_results", os.path.join(SRC, "glmnet_r_results.py"))
mod = importlib.util.module_from_spec(spec)
spec.loader.exec_module(mod)
cases = []
for name in sorted(x for x in dir(mod) if x.startswith("rslt_")):
    v = getattr(mod, name)
    if float(v[2]) != 0.0:
        continue  # ridge only
    cases.append(np.concatenate([v[:4], np.pad(v[4:], (0, 5 - (v.size - 4)))]))
np.savez(OUT, data=data, cases=np.array(cases))
print(OUT, len(cases), "cases")
