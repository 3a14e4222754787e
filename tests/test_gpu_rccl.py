"""RCCL on the one GPU of the test box (the loci-sharded path's partial-GRM all-reduce and the
distributed factorisation's strip all-gathers). A box has one GPU, so the collectives run on a 1-rank
communicator: the C ABI's GBM_FORCE_RCCL hook (ncclCommInitAll over device 0, ncclAllReduce of the packed
partial GRM, ncclAllGather of every distributable panel group's rows) and bench.py's `--collectives always`
(torch.distributed nccl = RCCL at world size 1). A sum or gather over one rank is the identity, so each run
must give the same bits as the run without collectives; the RCCL call counters prove the collectives ran."""
import ctypes
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import gbm
import oracle
from gbm import _lib

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / np.abs(np.asarray(b)).max())


def _rccl_calls():
    a, g = ctypes.c_int64(0), ctypes.c_int64(0)
    gbm.load_library().gbm_debug_rccl_calls(ctypes.byref(a), ctypes.byref(g))
    return a.value, g.value


@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_c_abi_forced_rccl_one_rank_bit_identical(gbm_env, devices):
    """gbm_gblup_fit with GBM_FORCE_RCCL=1: the packed partial GRM goes through ncclAllReduce and every
    distributable panel group's final rows through ncclAllGather (GBM_DIST_SOLVE_MIN_N / GBM_DIST_TAIL_ROWS = 0
    so that a 3 000-row fit has them) — bit-identical to the same fit without collectives (both on the
    launch-per-panel Cholesky, GBM_CHOL_FLOW_MAX = 0), and to the oracle within the parity bar."""
    n, p = 3000, 4000
    X = oracle.synth_genotypes(515, n, p)
    Y = oracle.synth_phenotypes(X, 16, ntraits=2)
    gbm_env.setenv("GBM_CHOL_FLOW_MAX", "0")
    gbm_env.setenv("GBM_DIST_SOLVE_MIN_N", "0")
    gbm_env.setenv("GBM_DIST_TAIL_ROWS", "0")
    ref_gpu = gbm.gblup_arrays(X, Y, lambda_=1.0, devices=devices, grm="fp64")
    a0, g0 = _rccl_calls()
    gbm_env.setenv("GBM_FORCE_RCCL", "1")
    forced = gbm.gblup_arrays(X, Y, lambda_=1.0, devices=devices, grm="fp64")
    a1, g1 = _rccl_calls()
    assert a1 - a0 == 1, (a0, a1)  # one partial-GRM all-reduce
    assert g1 - g0 >= 4, (g0, g1)  # one row all-gather per distributable group
    for x, y in zip(forced, ref_gpu):
        assert np.array_equal(np.asarray(x), np.asarray(y))
    ref = oracle.gblup_fit(X, Y, 1.0)
    assert forced[3] == ref["q"] and rel(forced[1], ref["y_pred"]) < 1e-9 and rel(forced[0], ref["b_hat"]) < 1e-6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _world1_worker(rank, port, n, p, seed, out_dir):
    sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))
    import torch
    import torch.distributed as dist

    from gbm import synth
    from gbm.sharded import HipShardStages, LocalComm, TorchComm, assemble_b_hat, sharded_gblup_step

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    from gbm import _lib
    _lib.debug_set("GBM_CHOL_FLOW_MAX", "0")
    st = HipShardStages(n, p, nrhs=1, lambda_=1.0, device=0)
    st.generate(seed, 0)
    Y = synth.qtl_phenotypes(seed, n, p, 1, device=0)
    st.load_phenotypes(Y)
    base = sharded_gblup_step(st, LocalComm())
    base = {k: np.array(v) for k, v in base.items()}
    _lib.debug_set("GBM_DIST_SOLVE_MIN_N", "0")
    _lib.debug_set("GBM_DIST_TAIL_ROWS", "0")
    comm = TorchComm(force=True)
    calls = {"all_reduce": 0, "all_gather": 0}
    ar, ag = comm.all_reduce_sum, comm.all_gather

    def count_ar(t):
        calls["all_reduce"] += 1
        return ar(t)

    def count_ag(t):
        calls["all_gather"] += 1
        return ag(t)

    comm.all_reduce_sum, comm.all_gather = count_ar, count_ag
    forced = sharded_gblup_step(st, comm)
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, "world1.npz"), **{"base_" + k: v for k, v in base.items()},
             **{"forced_" + k: np.array(v) for k, v in forced.items()}, Y=Y,
             b_hat=assemble_b_hat(forced["mu"], forced["msum"], [forced["B"]], p), backend=dist.get_backend(),
             n_all_reduce=calls["all_reduce"], n_all_gather=calls["all_gather"], world=dist.get_world_size())
    dist.destroy_process_group()


def test_torch_nccl_world1_forced_collectives_bit_identical(tmp_path):
    """sharded_gblup_step with TorchComm(force=True) over torch's nccl backend (RCCL) at world size 1 — what
    `bench.py --collectives always` runs — equals the step without collectives bit for bit, and the oracle."""
    import torch.multiprocessing as mp

    n, p, seed = 2500, 3000, 77
    mp.spawn(_world1_worker, args=(_free_port(), n, p, seed, str(tmp_path)), nprocs=1, join=True)
    r = dict(np.load(tmp_path / "world1.npz"))
    assert str(r["backend"]) == "nccl" and int(r["world"]) == 1
    assert int(r["n_all_reduce"]) == 2  # packed partial GRM + q, and the Σ m_j b_j partials
    assert int(r["n_all_gather"]) >= 3
    for k in ("B", "y_pred", "mu", "msum"):
        assert np.array_equal(r["base_" + k], r["forced_" + k]), k
    X = oracle.synth_genotypes(seed, n, p)
    ref = oracle.gblup_fit(X, r["Y"], 1.0)
    assert rel(r["forced_y_pred"], ref["y_pred"]) < 1e-9 and rel(r["b_hat"], ref["b_hat"]) < 1e-6


def test_bench_collectives_always_runs_rccl_at_one_rank():
    """`bench.py --collectives always` at N = 1: a 1-rank RCCL process group, the line records world_size 1,
    backend nccl and the per-rank stage times."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--collectives", "always", "--steps", "2", "--warmup", "1",
           "--individuals", "2000", "--loci", "6000", "--no-cpu-baseline", "--no-host-path", "--no-exact"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 1 and rec["world_size"] == 1 and rec["backend"] == "nccl"
    assert rec["collectives"].startswith("RCCL") and len(rec["per_rank_stage_ms"]) == 1
    assert rec["value"] > 0 and rec["stage_ms"]["allreduce"] > 0.0
