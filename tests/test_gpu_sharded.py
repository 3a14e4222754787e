"""N-rank loci sharding with the real HIP stages: 2 ranks on the one GPU of the test box, gloo
for the all-reduces (RCCL needs distinct devices per rank; the wiring is the same code path as
bench.py's nccl runs). Compares the assembled fit with the oracle on the full problem."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, p_total, seed, Y, out_dir, env=None):
    import sys
    os.environ.update(env or {})
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "genomicbreedingmodels.jl_amd"))
    import torch
    import torch.distributed as dist
    from gbm.sharded import HipExactShardStages, HipShardStages, TorchComm, sharded_gblup_step

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    per = (p_total + world - 1) // world
    j0 = rank * per
    p_local = min(per, p_total - j0)
    if os.environ.get("GBM_TEST_STAGES") == "exact":  # the exact-integer GRM shard (dosages resident)
        st = HipExactShardStages(n, p_local, nrhs=Y.shape[1], lambda_=1.0, device=0)
    else:
        st = HipShardStages(n, p_local, nrhs=Y.shape[1], lambda_=1.0, device=0)
    st.generate(seed, j0)
    st.load_phenotypes(Y)
    saved = {}

    def mark(label):  # the summed GRM, as the solve receives it
        if label == "allreduce":
            saved["G"], saved["q"] = st.G.clone(), st.q.clone()

    out = sharded_gblup_step(st, TorchComm(), events=mark)
    # the redundant launch-per-panel solve of the same summed G (the distributed factorisation computes
    # every tile with the same kernel and operands: the same bits)
    st.G.copy_(saved["G"])
    st.q.copy_(saved["q"])
    from gbm import _lib
    _lib.debug_set("GBM_CHOL_FLOW_MAX", "0")  # (libgbm read the environment at its first call)
    st.solve()
    torch.cuda.synchronize()
    y_red = st.gebv[:, :n].T.cpu().numpy()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **out, j0=j0, y_redundant=y_red)
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_one_gpu_match_oracle(tmp_path):
    import torch.multiprocessing as mp

    import oracle
    from gbm.sharded import assemble_b_hat

    n, p, seed = 400, 3001, 91
    X = oracle.synth_genotypes(seed, n, p)
    Y = oracle.synth_phenotypes(X, 5, ntraits=2)
    mp.spawn(_worker, args=(2, _free_port(), n, p, seed, Y, str(tmp_path)), nprocs=2, join=True)
    outs = [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(2)]
    ref = oracle.gblup_fit(X, Y, 1.0)
    for o in outs:
        assert np.abs(o["y_pred"] - ref["y_pred"]).max() < 1e-9 * np.abs(ref["y_pred"]).max()
    b_hat = assemble_b_hat(outs[0]["mu"], outs[0]["msum"], [o["B"] for o in outs], p)
    assert np.abs(b_hat - ref["b_hat"]).max() < 1e-6 * np.abs(ref["b_hat"]).max()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_ranks_one_gpu_distributed_solve_match_oracle(tmp_path, world):
    """The distributed factorisation (chol_distributed) over torch.distributed: each rank updates
    its own tile columns, strips all-gathered over gloo; forced on at a small n with 4-panel groups
    and a short redundant tail; world 8 = the north star's rank count (8 processes on the one GPU).
    Every rank's GEBVs equal the oracle's, and equal bit for bit the redundant solve of the same
    summed G."""
    import torch.multiprocessing as mp

    import oracle
    from gbm.sharded import assemble_b_hat

    n, p, seed = 1500, 2000, 17
    X = oracle.synth_genotypes(seed, n, p)
    Y = oracle.synth_phenotypes(X, 6, ntraits=2)
    env = {"GBM_DIST_SOLVE_MIN_N": "0", "GBM_DIST_TAIL_ROWS": "256", "GBM_CHOL_G4_LIM": "0",
           "GBM_CHOL_G8_LIM": "-1", "GBM_CHOL_G16_LIM": "-1", "GBM_UPD64_LIM": "128"}
    mp.spawn(_worker, args=(world, _free_port(), n, p, seed, Y, str(tmp_path), env), nprocs=world, join=True)
    outs = [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(world)]
    ref = oracle.gblup_fit(X, Y, 1.0)
    for o in outs:
        assert np.abs(o["y_pred"] - ref["y_pred"]).max() < 1e-9 * np.abs(ref["y_pred"]).max()
        assert np.array_equal(o["y_pred"], outs[0]["y_pred"])
        assert np.array_equal(o["y_pred"], o["y_redundant"])
    b_hat = assemble_b_hat(outs[0]["mu"], outs[0]["msum"], [o["B"] for o in outs], p)
    assert np.abs(b_hat - ref["b_hat"]).max() < 1e-6 * np.abs(ref["b_hat"]).max()


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_one_gpu_exact_grm_match_oracle(tmp_path, world):
    """Loci-sharded exact-integer GRMs (csrc/grm_exact.hip, each rank its own weights' fixed point) summed by
    the packed all-reduce, over gloo on the one GPU; the distributed factorisation forced on: the GEBVs and
    b_hat equal the oracle's fit of the whole problem."""
    import torch.multiprocessing as mp

    import oracle
    from gbm.sharded import assemble_b_hat

    n, p, seed = 700, 3001, 23
    X = oracle.synth_genotypes(seed, n, p)
    Y = oracle.synth_phenotypes(X, 4, ntraits=2)
    env = {"GBM_TEST_STAGES": "exact", "GBM_DIST_SOLVE_MIN_N": "0", "GBM_DIST_TAIL_ROWS": "256",
           "GBM_CHOL_G4_LIM": "0", "GBM_CHOL_G8_LIM": "-1", "GBM_CHOL_G16_LIM": "-1", "GBM_UPD64_LIM": "128"}
    mp.spawn(_worker, args=(world, _free_port(), n, p, seed, Y, str(tmp_path), env), nprocs=world, join=True)
    outs = [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(world)]
    ref = oracle.gblup_fit(X, Y, 1.0)
    for o in outs:
        assert np.abs(o["y_pred"] - ref["y_pred"]).max() < 1e-9 * np.abs(ref["y_pred"]).max()
    b_hat = assemble_b_hat(outs[0]["mu"], outs[0]["msum"], [o["B"] for o in outs], p)
    assert np.abs(b_hat - ref["b_hat"]).max() < 1e-6 * np.abs(ref["b_hat"]).max()


def test_bench_c3_leg_two_ranks_same_device():
    """bench.py's C3 leg at N = 2 on the one GPU of the test box (--same-device, gloo: RCCL
    needs one device per rank), on a reduced C3 (n = 20 000, 60 000 loci split 2 x 30 000, 15 000-locus chunks):
    the packed all-reduce and — n >= GBM_DIST_SOLVE_MIN_N = 16 384 — the distributed Cholesky run through the leg,
    both ranks end with the same GEBVs, q = p, and the record carries every rank's stage and collective times."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--same-device", "--dist-backend", "gloo",
           "--individuals", "2000", "--loci", "5000", "--steps", "1", "--warmup", "0", "--no-cpu-baseline",
           "--no-exact", "--no-host-path", "--c3-leg", "on", "--c3-individuals", "20000", "--c3-loci", "60000",
           "--c3-chunk", "15000", "--c3-steps", "1", "--c3-warmup", "1"]
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=root)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
    c3 = rec["c3"]
    print("\nC3 leg (reduced, 2 ranks on one GPU, gloo):", json.dumps(c3))
    assert c3["ranks"] == 2 and c3["n"] == 20000 and c3["p_total"] == 60000
    assert c3["ranks_agree"] and c3["q"] == 60000
    assert c3["value"] > 0 and 0 < c3["grm_frac_of_peak"] and 0 < c3["e2e_fp64_frac_of_peak"]
    for r in c3["per_rank"]:
        assert r["loci"] == 30000 and r["y_pred_finite"]
        assert r["allgather_calls"] > 0 and r["allgather_blocked_ms"] > 0  # the distributed solve engaged
        assert r["allreduce_bytes"] > 8 * 20000 * 20000 // 2  # the packed upper tiles (+ q) were all-reduced
    cx = rec["c3_exact_grm"]  # the same C3 with the exact-integer GRM: the same q, both ranks agree
    print("C3 leg, exact GRM:", json.dumps({k: v for k, v in cx.items() if k != "per_rank"}))
    assert cx["ranks"] == 2 and cx["digit_slices"] >= 8 and cx["value"] > 0
    assert {r["q"] for r in cx["per_rank"]} == {60000} and len({(r["y_pred_sum"], r["mu"]) for r in cx["per_rank"]}) == 1
    # the exact and fp64 GRMs give the same fit to rounding
    assert abs(cx["per_rank"][0]["mu"] - c3["per_rank"][0]["mu"]) < 1e-9 * abs(c3["per_rank"][0]["mu"])
