"""The N > 1 loci-sharded path on CPU: world_size 2 over gloo drives the same
``sharded_gblup_step`` (and the same all-reduce wiring) that bench.py runs over RCCL, with a
numpy stage backend standing in for the HIP stages (test infrastructure, not the product)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from gbm.sharded import TorchComm, assemble_b_hat, sharded_gblup_step


class NumpyShardStages:
    """Stage semantics of gbm.sharded.HipShardStages restated with numpy on torch CPU tensors."""

    def __init__(self, X_local, Y, lam):
        self.X = X_local
        self.Y = Y
        self.lam = lam
        n = X_local.shape[0]
        self.G = torch.zeros((n, n), dtype=torch.float64)
        self.q = torch.zeros(1, dtype=torch.int64)
        self.msum = torch.zeros(Y.shape[1], dtype=torch.float64)

    def standardize(self):
        self.m, self.s, self.keep = oracle.colstats(self.X)
        self.Z = oracle.standardize(self.X, self.m, self.s, self.keep)
        self.q.fill_(int(self.keep.sum()))

    def grm_syrk(self):
        self.G.copy_(torch.from_numpy(self.Z @ self.Z.T))

    def grm_reduce(self):
        pass

    def grm_rows(self):
        return self.G

    def solve(self):
        import scipy.linalg as sla
        n = self.X.shape[0]
        q = int(self.q.item())
        V = self.G.numpy() / q + self.lam * np.eye(n)
        c = sla.cho_factor(V, lower=True)
        one = np.ones(n)
        mu = (one @ sla.cho_solve(c, self.Y)) / (one @ sla.cho_solve(c, one))
        self.mu = mu
        self.A = sla.cho_solve(c, self.Y - mu)
        self.y_pred = mu + (self.Y - mu) - self.lam * self.A

    def effects(self):
        q = int(self.q.item())
        B = np.zeros((self.Y.shape[1], self.X.shape[1]))
        B[:, self.keep] = ((self.Z.T @ self.A) / q / self.s[self.keep][:, None]).T
        self.B = B
        self.msum.copy_(torch.from_numpy(B @ self.m))

    def download(self):
        return dict(B=self.B, y_pred=self.y_pred, mu=self.mu, msum=self.msum.numpy().copy())


def _worker(rank, world, port, X, Y, lam, out_dir):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    p = X.shape[1]
    per = (p + world - 1) // world
    j0, j1 = rank * per, min(p, (rank + 1) * per)
    st = NumpyShardStages(X[:, j0:j1], Y, lam)
    out = sharded_gblup_step(st, TorchComm())
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **out, j0=j0)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_step_gloo_matches_full_problem(tmp_path, world):
    n, p = 90, 301  # p not divisible by world
    X = oracle.synth_genotypes(31, n, p)
    X[:, 7] = 0.5  # a monomorphic locus inside shard 0
    Y = oracle.synth_phenotypes(X, 6, ntraits=2)
    lam = 0.7
    mp.spawn(_worker, args=(world, _free_port(), X, Y, lam, str(tmp_path)), nprocs=world, join=True)
    outs = [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(world)]
    ref = oracle.gblup_fit(X, Y, lam)
    for o in outs:  # every rank holds the same GEBVs and μ̂
        assert np.abs(o["y_pred"] - ref["y_pred"]).max() < 1e-10 * np.abs(ref["y_pred"]).max()
        assert np.abs(o["mu"] - ref["mu"]).max() < 1e-10
    b_hat = assemble_b_hat(outs[0]["mu"], outs[0]["msum"], [o["B"] for o in outs], p)
    assert np.abs(b_hat - ref["b_hat"]).max() < 1e-9 * np.abs(ref["b_hat"]).max()
    assert b_hat[1 + 7, 0] == 0.0
