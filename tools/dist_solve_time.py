"""Per-rank cost of the distributed GBLUP factorisation at a C3-like n, on one GPU: rank 0 of R
runs every panel group's panels and trailing update on its own tiles (plus the group's diagonal
area and the right-hand sides) and both per-group exchanges' pack/unpack; the all-gather is
replaced by R copies of its own pack (wrong values for the other ranks' columns, so only the timing
is meaningful). Prints the redundant single-rank solve, the per-rank solve for each R, and the bytes
each rank would receive per solve. Timing tool only.
Usage: python tools/dist_solve_time.py [n] [R ...]   (SKIP_REDUNDANT=1: the distributed solves only)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gbm.sharded import HipShardStages, chol_distributed  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
Rs = [int(a) for a in sys.argv[2:]] or [8, 4, 2]
p = 2000  # any SPD G times the same
st = HipShardStages(n, p, nrhs=1, lambda_=1.0, device=0)
st.generate(424242, 0)
st.load_phenotypes(np.random.default_rng(0).standard_normal(n))
st.standardize()
st.grm_syrk()
st.grm_reduce()
G0 = st.G.clone()
torch.cuda.synchronize()


def timed(fn, reps=2):
    ts = []
    for _ in range(reps + 1):
        st.G.copy_(G0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts[1:])


res = {"n": n}
if not os.environ.get("SKIP_REDUNDANT"):  # (a kernel trace of the distributed solve alone)
    res["redundant_solve_s"] = timed(st.solve)
for R in Rs:
    recv = [0]

    def allgather(packs, R=R):
        recv[0] += packs[0].numel() * 8 * (R - 1)
        return [torch.cat([packs[0]] * R)]

    t = timed(lambda: chol_distributed([st], [0], R, allgather))
    res[f"R{R}"] = {"per_rank_solve_s": t, "bytes_received_per_rank": recv[0] // 3}
print(json.dumps(res), flush=True)
