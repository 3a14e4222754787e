"""The N > 1 loci-sharded path on CPU: world sizes 2, 3 and 8 (the north star's rank count) over
gloo drive the same ``sharded_gblup_step`` / ``chol_distributed`` (and the same collective wiring)
that bench.py runs over RCCL, with a numpy stage backend standing in for the HIP stages (test
infrastructure, not the product). The backend restates the stage semantics of gbm.sharded.
HipShardStages at tile level: the packed partial-GRM all-reduce (upper 128-tiles + q in the last
slot) and the distributed factorisation protocol of gbm_dev_chol_* (include/gbm.h): per panel group
the group's diagonal area is all-gathered (its columns' owners updated them) and its first block
factored, every rank runs the group's panels and row updates on its own 128-column tiles (J ≡ rank
mod R), the area and the bordered right-hand sides, the group's rows are all-gathered, and the
trailing update runs on the rank's own tiles and the right-hand sides; the tail runs redundantly. Every tile update is the same numpy op
whichever rank computes it, so the distributed solve equals the redundant one bit for bit."""
import contextlib
import os
import socket

import numpy as np
import pytest
import scipy.linalg as sla
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from gbm.sharded import TorchComm, assemble_b_hat, sharded_gblup_step

NB, TB = 64, 128  # panel rows, ownership tile columns (csrc: kCholNB, the GRM tile)


class _NumpyChol:
    """gbm_dev_chol_group_size for the numpy backend: 4-panel groups while more than 6 blocks remain,
    then 2-panel groups, then single panels (groups of >= 2 panels starting on a 128-row boundary
    are distributable, as in csrc/chol.hip)."""

    def __init__(self, npad):
        self.nb = npad // NB

    def gbm_dev_chol_group_size(self, n, kb):
        rem = self.nb - kb
        return 0 if rem <= 0 else 4 if rem > 6 else 2 if rem > 2 else 1


class NumpyShardStages:
    """Stage semantics of gbm.sharded.HipShardStages restated with numpy on torch CPU tensors."""

    def __init__(self, X_local, Y, lam):
        self.X = X_local
        self.Y = Y
        self.lam = lam
        n = X_local.shape[0]
        self.n = n
        self.npad = -(-n // TB) * TB
        self.gdim = self.npad + NB
        self.lib = _NumpyChol(self.npad)
        self.G = torch.zeros((self.gdim, self.gdim), dtype=torch.float64)
        self.q = torch.zeros(1, dtype=torch.int64)
        self.msum = torch.zeros(Y.shape[1], dtype=torch.float64)
        self.packs = 0

    def standardize(self):
        self.m, self.s, self.keep = oracle.colstats(self.X)
        self.Z = oracle.standardize(self.X, self.m, self.s, self.keep)
        self.q.fill_(int(self.keep.sum()))

    def grm_syrk(self):
        self.G[: self.n, : self.n] = torch.from_numpy(self.Z @ self.Z.T)

    def grm_reduce(self):
        pass

    def grm_rows(self):
        return self.G[: self.npad]

    # ---- the packed all-reduce operand: upper 128-tiles of G, then q (gbm_dev_grm_pack) ----------
    def _tiles(self):
        nt = self.npad // TB
        return [(i, j) for i in range(nt) for j in range(i, nt)]

    def grm_pack(self):
        self.packs += 1
        parts = [self.G[i * TB:(i + 1) * TB, j * TB:(j + 1) * TB].reshape(-1) for i, j in self._tiles()]
        self.Gp = torch.cat(parts + [self.q.to(torch.float64)])
        return self.Gp

    def grm_unpack(self):
        for k, (i, j) in enumerate(self._tiles()):
            self.G[i * TB:(i + 1) * TB, j * TB:(j + 1) * TB] = self.Gp[k * TB * TB:(k + 1) * TB * TB].view(TB, TB)
        self.q.fill_(int(self.Gp[-1].item()))

    # ---- the solve in phases (gbm_dev_chol_prepare / group_panels / strip_pack / strip_unpack_rows /
    # group_update / area_pack / area_unpack / strip_unpack / factor_diag / group /
    # finish): V = G/q + λI bordered by R = [1, y...], upper factor U, W = U⁻ᵀR in the border ---------
    def chol_prepare(self):
        n, npad, t = self.n, self.npad, self.Y.shape[1]
        V = np.zeros((self.gdim, self.gdim))
        V[:n, :n] = np.triu(self.G[:n, :n].numpy()) / int(self.q.item())
        V[np.arange(n), np.arange(n)] += self.lam
        V[np.arange(n, npad), np.arange(n, npad)] = 1.0
        V[:n, npad] = 1.0
        V[:n, npad + 1:npad + 1 + t] = self.Y
        self.V = V
        self.chol_factor_diag(0)

    def chol_prepare_cols(self, rank, nranks):
        """gbm_dev_chol_prepare_cols: V on the rank's own tiles, the first group's area and the right-hand
        sides only; every other column keeps G (its rows arrive by exchanges before they are read)."""
        self.chol_prepare()
        g0 = self.lib.gbm_dev_chol_group_size(self.n, 0)
        raw = np.zeros_like(self.V)
        raw[:self.n, :self.n] = np.triu(self.G[:self.n, :self.n].numpy())
        for c in range(self.npad):
            if not (c < NB * g0 or (c // TB) % nranks == rank):
                self.V[:, c] = raw[:, c]

    def chol_factor_diag(self, kb):
        r = slice(NB * kb, NB * kb + NB)
        A = np.triu(self.V[r, r])
        self.V[r, r] = np.linalg.cholesky(A + np.triu(A, 1).T).T

    def _chunks(self, c_lo, keep):
        """The 128-tile column chunks of [c_lo, npad) that ``keep`` selects, then the right-hand sides
        (every rank's). Both the redundant and the distributed solve apply each op chunk by chunk, so
        a chunk's bits do not depend on which rank computes it."""
        out, c = [], c_lo
        while c < self.npad:
            c1 = min((c // TB + 1) * TB, self.npad)
            if keep(c):
                out.append(slice(c, c1))
            c = c1
        return out + [slice(self.npad, self.gdim)]

    def chol_group_panels(self, kb, rank, nranks):
        """The group's panels and row updates on the kept columns: the rank's own tiles, the group's
        diagonal area (< keep_hi) and the right-hand sides (gbm_dev_chol_group_panels)."""
        V = self.V
        g = self.lib.gbm_dev_chol_group_size(self.n, kb)
        keep_hi = NB * (kb + g)
        chunks = lambda lo: self._chunks(lo, lambda c: nranks == 1 or c < keep_hi or (c // TB) % nranks == rank)
        for k in range(kb, kb + g):
            r = slice(NB * k, NB * k + NB)
            if k > kb:  # this group's earlier panels
                for ch in chunks(NB * k):
                    for pj in range(kb, k):
                        rp = slice(NB * pj, NB * pj + NB)
                        V[r, ch] -= V[rp, r].T @ V[rp, ch]
                self.chol_factor_diag(k)
            for ch in chunks(NB * (k + 1)):
                V[r, ch] = sla.solve_triangular(V[r, r], V[r, ch], trans="T", lower=False)

    def chol_group_update(self, kb, rank, nranks, col_lo=0, col_hi=None, row_lo=0, row_hi=None):
        """The trailing update on the rank's own tiles and the right-hand sides; on one rank the next
        diagonal block is factored too (gbm_dev_chol_group_update). col_lo/col_hi: the rank's tiles
        with columns in [col_lo, col_hi), the right-hand sides when col_hi >= gdim
        (gbm_dev_chol_group_update_cols); row_lo/row_hi: the rows [row_lo, row_hi) of those tiles
        (gbm_dev_chol_group_update_tiles)."""
        V, npad, nb = self.V, self.npad, self.npad // NB
        g = self.lib.gbm_dev_chol_group_size(self.n, kb)
        k0, k1 = NB * kb, NB * (kb + g)
        col_hi = self.gdim if col_hi is None else col_hi
        row_hi = self.gdim if row_hi is None else row_hi
        keep = lambda c: (nranks == 1 or (c // TB) % nranks == rank) and col_lo <= c < col_hi
        for ch in self._chunks(k1, keep):
            if ch.start >= npad and col_hi < self.gdim:
                continue  # the right-hand sides belong to the call that reaches gdim
            r0, rend = max(k1, row_lo), min(ch.stop, npad, row_hi)
            if rend > r0:
                V[r0:rend, ch] -= V[k0:k1, r0:rend].T @ V[k0:k1, ch]
        if nranks == 1 and kb + g < nb:
            self.chol_factor_diag(kb + g)

    def chol_group_update_cols(self, kb, rank, nranks, col_lo, col_hi):
        self.chol_group_update(kb, rank, nranks, col_lo, col_hi)

    def chol_group_update_tiles(self, kb, rank, nranks, row_lo, row_hi, col_lo, col_hi):
        self.chol_group_update(kb, rank, nranks, col_lo, col_hi, row_lo, row_hi)

    # the overlap hooks of chol_distributed (streams on the GPU; here the calls run in order)
    def fork(self):
        pass

    def side(self):
        return contextlib.nullcontext()

    def join(self):
        pass

    def lower_fork(self):
        pass

    def lower(self):
        return contextlib.nullcontext()

    def lower_join(self):
        pass

    def chol_lower_copy(self, kb, rows64, rank, nranks):
        pass  # (V holds the upper factor only: strip_unpack and strip_unpack_rows are the same here)

    def chol_group(self, kb, rank, nranks):
        assert (rank, nranks) == (0, 1)  # gbm_dev_chol_group: the redundant path only
        self.chol_group_panels(kb, 0, 1)
        self.chol_group_update(kb, 0, 1)

    def _owned_cols(self, kb, rank, nranks, end=None):
        c = np.arange(NB * kb, self.npad if end is None else end)
        return c[(c // TB) % nranks == rank]

    def _strip_doubles(self, kb, rows64, nranks, end=None):
        """Per-rank pack size, padded to the largest rank's (gbm_dev_chol_strip_doubles): the
        all-gather moves equal pieces."""
        return NB * rows64 * max(self._owned_cols(kb, r, nranks, end).size for r in range(nranks))

    def strip_pack(self, kb, rows64, rank, nranks, end=None):
        rows = slice(NB * kb, NB * (kb + rows64))
        buf = np.zeros(self._strip_doubles(kb, rows64, nranks, end))
        own = np.ascontiguousarray(self.V[rows][:, self._owned_cols(kb, rank, nranks, end)]).ravel()
        buf[:own.size] = own
        return torch.from_numpy(buf)

    def strip_unpack(self, kb, rows64, nranks, gathered, end=None):
        rows = slice(NB * kb, NB * (kb + rows64))
        g = gathered.numpy()
        per = self._strip_doubles(kb, rows64, nranks, end)
        for r in range(nranks):
            cols = self._owned_cols(kb, r, nranks, end)
            self.V[rows, cols] = g[r * per:r * per + NB * rows64 * cols.size].reshape(NB * rows64, cols.size)

    def area_pack(self, kb, rows64, rank, nranks):  # the square diagonal area (gbm_dev_chol_area_pack)
        return self.strip_pack(kb, rows64, rank, nranks, end=NB * (kb + rows64))

    def area_unpack(self, kb, rows64, nranks, gathered):
        self.strip_unpack(kb, rows64, nranks, gathered, end=NB * (kb + rows64))

    def strip_unpack_rows(self, kb, rows64, rank, nranks, gathered):
        self.strip_unpack(kb, rows64, nranks, gathered)  # (the lower copy is not modelled: finish reads triu)

    def chol_finish(self):
        n, npad, t = self.n, self.npad, self.Y.shape[1]
        U = np.triu(self.V[:npad, :npad])
        W = self.V[:npad, npad:npad + 1 + t]
        w1, wy = W[:, 0], W[:, 1:]
        mu = (w1 @ wy) / (w1 @ w1)
        self.mu = mu
        self.A = sla.solve_triangular(U, wy - np.outer(w1, mu), lower=False)[:n]
        self.y_pred = mu + (self.Y - mu) - self.lam * self.A

    def solve(self):
        """The redundant solve: the same phases on one rank (every tile owned)."""
        self.chol_prepare()
        kb, nb = 0, self.npad // NB
        while kb < nb:
            g = self.lib.gbm_dev_chol_group_size(self.n, kb)
            self.chol_group(kb, 0, 1)
            kb += g
        self.chol_finish()

    def effects(self):
        q = int(self.q.item())
        B = np.zeros((self.Y.shape[1], self.X.shape[1]))
        B[:, self.keep] = ((self.Z.T @ self.A) / q / self.s[self.keep][:, None]).T
        self.B = B
        self.msum.copy_(torch.from_numpy(B @ self.m))

    def download(self):
        return dict(B=self.B, y_pred=self.y_pred, mu=self.mu, msum=self.msum.numpy().copy())


def _worker(rank, world, port, X, Y, lam, out_dir, env=None):
    os.environ.update(env or {})
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    p = X.shape[1]
    per = (p + world - 1) // world
    j0, j1 = rank * per, min(p, (rank + 1) * per)
    st = NumpyShardStages(X[:, j0:j1], Y, lam)
    saved = {}

    def mark(label):  # the summed GRM, as the solve receives it
        if label == "allreduce":
            saved["G"], saved["q"] = st.G.clone(), st.q.clone()

    out = sharded_gblup_step(st, TorchComm(force=os.environ.get("GBM_TEST_FORCE") == "1"), events=mark)
    # the redundant solve on the same summed G (what one rank alone computes from it)
    st.G.copy_(saved["G"])
    st.q.copy_(saved["q"])
    st.solve()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **out, j0=j0, y_redundant=st.y_pred, packs=st.packs)
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


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_step_gloo_distributed_solve_bit_identical(tmp_path, world):
    """World size 8 as on the north star's 8-GPU node (and 2): packed partial-GRM all-reduce, then the
    distributed factorisation forced on at a small n (GBM_DIST_SOLVE_MIN_N = 0, a 128-row redundant
    tail): 4- and 2-panel groups distributed over the ranks' tile columns (with 8 ranks and 5 tile
    columns, three ranks own none), each group's rows all-gathered over gloo, the tail redundant. Each rank's
    distributed solve equals the redundant solve of the same summed G bit for bit, every rank holds
    the same GEBVs, and the assembled fit matches the oracle on the full problem."""
    n, p = 600, 1500
    X = oracle.synth_genotypes(77, n, p)
    Y = oracle.synth_phenotypes(X, 8, ntraits=2)
    lam = 0.9
    env = {"GBM_DIST_SOLVE_MIN_N": "0", "GBM_DIST_TAIL_ROWS": "128"}
    mp.spawn(_worker, args=(world, _free_port(), X, Y, lam, str(tmp_path), env), nprocs=world, join=True)
    outs = [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(world)]
    ref = oracle.gblup_fit(X, Y, lam)
    for o in outs:
        assert int(o["packs"]) == 1  # the packed all-reduce ran
        assert np.array_equal(o["y_pred"], o["y_redundant"])
        assert np.array_equal(o["y_pred"], outs[0]["y_pred"])
    assert np.abs(outs[0]["y_pred"] - ref["y_pred"]).max() < 1e-10 * np.abs(ref["y_pred"]).max()
    b_hat = assemble_b_hat(outs[0]["mu"], outs[0]["msum"], [o["B"] for o in outs], p)
    assert np.abs(b_hat - ref["b_hat"]).max() < 1e-9 * np.abs(ref["b_hat"]).max()


def test_world1_forced_collectives_bit_identical(tmp_path):
    """bench.py --collectives always at one rank (TorchComm(force=True), here over gloo): the packed
    all-reduce and, with the distributed solve forced on, chol_distributed's one-rank branch (every
    distributable group's rows through the all-gather between its panels and its update) — the same bits
    as the redundant solve, and the oracle's fit."""
    n, p = 600, 1500
    X = oracle.synth_genotypes(78, n, p)
    Y = oracle.synth_phenotypes(X, 9, ntraits=2)
    lam = 1.1
    env = {"GBM_DIST_SOLVE_MIN_N": "0", "GBM_DIST_TAIL_ROWS": "0", "GBM_TEST_FORCE": "1"}
    mp.spawn(_worker, args=(1, _free_port(), X, Y, lam, str(tmp_path), env), nprocs=1, join=True)
    o = dict(np.load(tmp_path / "rank0.npz"))
    assert int(o["packs"]) == 1  # the all-reduce ran at world size 1
    assert np.array_equal(o["y_pred"], o["y_redundant"])
    ref = oracle.gblup_fit(X, Y, lam)
    assert np.abs(o["y_pred"] - ref["y_pred"]).max() < 1e-10 * np.abs(ref["y_pred"]).max()
