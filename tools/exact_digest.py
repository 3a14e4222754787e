"""Hash of the exact-integer GRM's G (upper n x n) through the stage API, for comparing builds
(GBM_LIBGBM=...): the class layout of the loci must not change a bit. Timing/check tool only."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gbm.sharded import HipExactShardStages  # noqa: E402

out = []
for n, p, seed in [(5000, 50000, 4242), (1030, 1234, 7), (777, 3001, 11), (2048, 20000, 3)]:
    st = HipExactShardStages(n, p, device=0)
    st.generate(seed, 0)
    st.standardize()
    st.grm_syrk()
    st.grm_reduce()
    torch.cuda.synchronize()
    G = np.triu(st.G[:n, :n].cpu().numpy())
    out.append(f"{n}x{p}:{hashlib.sha256(G.tobytes()).hexdigest()[:12]}")
    del st
    torch.cuda.empty_cache()
print(os.path.basename(os.environ.get("GBM_LIBGBM", "libgbm.so")), " ".join(out), flush=True)
