"""Loci-sharded GBLUP step for one-process-per-GPU runs (torch.distributed over RCCL/xGMI).

Each rank owns a contiguous block of loci (SNP columns) resident in its GPU's HBM. One step is

    standardise (local) → partial GRM Σ_j z_j z_jᵀ (local, fp64 MFMA)
      → all-reduce(sum) of the partial GRMs and of the kept-loci counts q      [RCCL]
      → GBLUP solve on G/q + λI: at large n a distributed Cholesky (each rank the trailing
        updates of its own 128-column tiles, a strip all-gather per panel group; chol_distributed),
        otherwise every rank redundantly (a stays local either way)
      → marker effects b_j for the rank's loci and Σ m_j b_j partials
      → all-reduce(sum) of the Σ m_j b_j partials (b0 = μ̂ − Σ)                 [RCCL]
      → results to the host.

The only data-path exchange is the partial-GRM all-reduce; the two others are
n_traits-sized scalars. ``sharded_gblup_step`` is written against two small interfaces so the
collective wiring is tested on CPU with gloo (tests/test_sharded_gloo.py): ``stages`` (the
HIP implementation is ``HipShardStages`` below) and ``comm``.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib


class TorchComm:
    """Sum all-reduce over torch.distributed (RCCL for cuda tensors, gloo for CPU tensors).

    ``force``: run every collective of the step even at world size 1 (``bench.py --collectives always``:
    the partial-GRM all-reduce and the Cholesky strip all-gathers execute on a 1-rank RCCL communicator,
    so the RCCL path runs on a one-GPU box; the results are the same bits as without collectives)."""

    def __init__(self, force: bool = False):
        import torch.distributed as dist
        self.dist = dist
        self.world_size = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.force = bool(force) and dist.is_initialized()

    def all_reduce_sum(self, t):
        if self.world_size > 1 or self.force:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)

    def all_gather(self, t):
        """Every rank's t, concatenated in rank order (one flat tensor)."""
        import torch
        out = torch.empty(self.world_size * t.numel(), dtype=t.dtype, device=t.device)
        if self.dist.get_backend() == "nccl":
            self.dist.all_gather_into_tensor(out, t.reshape(-1))
        else:  # gloo: list form
            parts = list(out.chunk(self.world_size))
            self.dist.all_gather(parts, t.reshape(-1).contiguous())
        return out


class LocalComm:
    world_size = 1
    rank = 0
    force = False

    def all_reduce_sum(self, t):
        return None


def sharded_gblup_step(stages, comm, events=None):
    """One GBLUP pass over the rank's shard. ``events`` (optional) is a callable(label) that
    records a timing mark on the compute stream between stages."""
    mark = events or (lambda label: None)
    mark("begin")
    stages.standardize()
    mark("standardize")
    stages.grm_syrk()
    mark("grm_syrk")
    stages.grm_reduce()
    mark("grm_reduce")
    collective = comm.world_size > 1 or getattr(comm, "force", False)
    if collective:
        # the upper GRM tiles only (half of G's rows) with q in the packed buffer's last slot (one
        # collective instead of two), when the stages can pack them
        pack = getattr(stages, "grm_pack", None)
        if pack is not None:
            comm.all_reduce_sum(pack())
            stages.grm_unpack()
        else:
            comm.all_reduce_sum(stages.grm_rows())
            comm.all_reduce_sum(stages.q)
    mark("allreduce")
    if collective and hasattr(stages, "chol_group") and stages.n >= dist_solve_min_n():
        chol_distributed([stages], [comm.rank], comm.world_size, lambda packs: [comm.all_gather(packs[0])],
                         force=getattr(comm, "force", False))
    else:
        stages.solve()
    mark("solve")
    stages.effects()
    comm.all_reduce_sum(stages.msum)
    mark("effects")
    out = stages.download()
    mark("download")
    return out


_SIDE_STREAMS = {}  # device -> the distributed solve's side stream
_LOWER_STREAMS = {}  # device -> the stream of its deferred lower copies


def dist_solve_min_n() -> int:
    """Individuals from which a multi-rank step factors V distributed (below, the latency-bound
    solve is cheaper redundantly). GBM_DIST_SOLVE_MIN_N overrides (tests)."""
    import os
    return int(os.environ.get("GBM_DIST_SOLVE_MIN_N", "16384"))


def chol_distributed(stages, ranks, nranks, allgather, tail_rows=None, force=False):
    """GBLUP solve of V = G/q + λI distributed over ``nranks`` ranks, replacing the
    redundant per-rank factorisation (the reference's pinv(V), src/gwas.jl:472,595).

    ``stages``: the ranks this process drives (HipShardStages, each holding the full summed G) —
    one in the one-process-per-GPU run, all of them in a single-process rehearsal; ``ranks``: their
    rank ids; ``allgather(packs)``: one packed strip per local rank -> per local rank the flat
    concatenation of all ranks' packs. Per panel group: after an earlier distributed group the
    group's diagonal area is all-gathered (its columns were updated by their owners) and its first
    block factored; every rank runs the group's panels and row updates on its own 128-column tiles
    (plus the area and the right-hand sides; gbm_dev_chol_group_panels), the group's solved rows are
    all-gathered (strip_unpack_rows also writes their lower copy), then the trailing update runs on
    the rank's own tiles and the right-hand sides (gbm_dev_chol_group_update). With overlap
    (GBM_DIST_OVERLAP, default 1; stages with fork/side/join), the next group's area is updated and
    exchanged on a side stream while the rest of the update runs (gbm_dev_chol_group_update_cols); with
    look-ahead (GBM_DIST_LOOKAHEAD, default 1) the next group's rows are updated first and its panels and
    row exchange run on the side stream too, beside the rest of the update
    (gbm_dev_chol_group_update_tiles).
    Once the trailing matrix is small (``tail_rows``, GBM_DIST_TAIL_ROWS, default 8192) or the groups
    shrink to single panels, every remaining row is gathered once and the tail runs redundantly. The
    result is bit-identical to the redundant solve (the same kernels compute every tile).

    ``nranks == 1`` with ``force`` (a 1-rank communicator: ``bench.py --collectives always``, the C ABI's
    GBM_FORCE_RCCL): the redundant solve, with each distributable group's final rows passed through the
    all-gather between its panels and its trailing update (an identity exchange on one rank), so the
    strip all-gather executes with real payloads; same bits as the redundant solve."""
    import os
    st0 = stages[0]
    lib, n = st0.lib, st0.n
    nb = st0.npad // 64
    gdim = st0.gdim
    if tail_rows is None:
        tail_rows = int(os.environ.get("GBM_DIST_TAIL_ROWS", "8192"))

    def distributable(kb):  # (a group reaching the end is the dataflow tail, GBM_CHOL_TAIL_FLOW)
        g = lib.gbm_dev_chol_group_size(n, kb)
        return gdim - 64 * kb > tail_rows and 2 <= g < nb - kb and (64 * kb) % 128 == 0

    overlap = int(os.environ.get("GBM_DIST_OVERLAP", "1")) != 0 and all(hasattr(st, "fork") for st in stages)

    defer_lower = all(hasattr(st, "lower_fork") for st in stages)

    def exchange(kb, rows64, what):  # "rows": a group's final rows; "rest": the tail; "area": a group's area
        # "rows_deferred": the final rows without their lower copy (the caller queues it on the lower stream)
        pack = "area_pack" if what == "area" else "strip_pack"
        packs = [getattr(st, pack)(kb, rows64, r, nranks) for st, r in zip(stages, ranks)]
        for st, r, gathered in zip(stages, ranks, allgather(packs)):
            if what == "rows":
                st.strip_unpack_rows(kb, rows64, r, nranks, gathered)
                continue
            if what == "rows_deferred":
                st.strip_unpack(kb, rows64, nranks, gathered)
                continue
            if what == "area":
                st.area_unpack(kb, rows64, nranks, gathered)
            else:
                st.strip_unpack(kb, rows64, nranks, gathered)
            st.chol_factor_diag(kb)

    if nranks > 1 and distributable(0):
        for st, r in zip(stages, ranks):  # V on the columns this rank reads before an exchange only
            st.chol_prepare_cols(r, nranks)
    else:
        for st in stages:
            st.chol_prepare()
    if nranks == 1 and force:
        kb = 0
        while kb < nb:
            g = int(lib.gbm_dev_chol_group_size(n, kb))
            if distributable(kb):
                for st, r in zip(stages, ranks):
                    st.chol_group_panels(kb, r, 1)
                exchange(kb, g, "rows")
                for st, r in zip(stages, ranks):
                    st.chol_group_update(kb, r, 1)
            else:
                for st in stages:
                    st.chol_group(kb, 0, 1)
            kb += g
        for st in stages:
            st.chol_finish()
        return
    lookahead = overlap and int(os.environ.get("GBM_DIST_LOOKAHEAD", "1")) != 0
    kb = 0
    dist = nranks > 1 and distributable(0)
    stale = False  # a distributed update skipped other ranks' tiles
    pending = False  # this group's area (look-ahead: also its panels and rows) is on the side stream
    ahead = False  # (look-ahead) this group's panels and row exchange were issued on the side stream
    while kb < nb:
        g = int(lib.gbm_dev_chol_group_size(n, kb))
        if not dist:
            for st in stages:
                st.chol_group(kb, 0, 1)
            kb += g
            continue
        if pending:
            for st in stages:
                st.join()
            pending = False
        elif stale:
            exchange(kb, g, "area")
        if not ahead:
            for st, r in zip(stages, ranks):
                st.chol_group_panels(kb, r, nranks)
            exchange(kb, g, "rows")
        ahead = False
        k1 = kb + g
        next_dist = k1 < nb and distributable(k1)
        if overlap and next_dist:
            g1 = int(lib.gbm_dev_chol_group_size(n, k1))
            area_hi = 64 * (k1 + g1)
            for st in stages:
                st.fork()
            if lookahead:
                # look-ahead: on the side stream the next group's rows of every kept column (its area among
                # them: one launch), the area exchange, its panels and its row exchange, beside the rest of
                # the update on this one (rows from area_hi on: disjoint tiles)
                with stages[0].side():
                    for st, r in zip(stages, ranks):
                        st.chol_group_update_tiles(kb, r, nranks, 64 * k1, area_hi, 64 * k1, gdim)
                    exchange(k1, g1, "area")
                    for st, r in zip(stages, ranks):
                        st.chol_group_panels(k1, r, nranks)
                    exchange(k1, g1, "rows_deferred" if defer_lower else "rows")
                    if defer_lower:
                        # the rows' lower copy (read only by chol_finish) off the side stream: the next join
                        # does not wait for it
                        for st in stages:
                            st.lower_fork()
                        with stages[0].lower():
                            for st, r in zip(stages, ranks):
                                st.chol_lower_copy(k1, g1, r, nranks)
                for st, r in zip(stages, ranks):
                    st.chol_group_update_tiles(kb, r, nranks, area_hi, gdim, area_hi, gdim)
                ahead = True
            else:
                # the next group's area (a rank owns about one of its tile columns: a few workgroups, one
                # K = 64 g tile long) is updated and exchanged on the side stream, beside the rest
                with stages[0].side():  # (one side stream per device)
                    for st, r in zip(stages, ranks):
                        st.chol_group_update_cols(kb, r, nranks, 64 * k1, area_hi)
                    exchange(k1, g1, "area")
                for st, r in zip(stages, ranks):
                    st.chol_group_update_cols(kb, r, nranks, area_hi, gdim)
            pending = True
        else:
            for st, r in zip(stages, ranks):
                st.chol_group_update(kb, r, nranks)
        stale = True
        kb = k1
        if kb >= nb:
            break
        dist = next_dist
        if not dist:  # the tail: every remaining row, once
            exchange(kb, nb - kb, "rest")
    for st in stages:
        if defer_lower:
            st.lower_join()  # the deferred lower copies, which the back substitution reads
        st.chol_finish()


def assemble_b_hat(mu, msum, B_shards, p_total):
    """b_hat (p+1, t): [μ̂ − Σ m_j b_j; b] (intercept first, reference src/linear.jl:218-221)."""
    t = len(mu)
    b_hat = np.zeros((p_total + 1, t))
    b_hat[0] = np.asarray(mu) - np.asarray(msum)
    off = 0
    for B in B_shards:
        b_hat[1 + off:1 + off + B.shape[1]] = B.T
        off += B.shape[1]
    return b_hat


class HipShardStages:
    """Device-resident buffers of one shard (torch-allocated HBM) driven through libgbm's
    stream-ordered C ABI on torch's current stream."""

    def __init__(self, n: int, p_local: int, nrhs: int = 1, lambda_: float = 1.0, device: int = 0):
        import torch
        self.torch = torch
        self.lib = _lib.load()
        self.n, self.p, self.nrhs, self.lam = n, p_local, nrhs, float(lambda_)
        self.dev = torch.device("cuda", device)
        lib = self.lib
        self.npad = lib.gbm_dev_npad(n)
        self.gdim = lib.gbm_dev_gdim(n)
        f64 = dict(dtype=torch.float64, device=self.dev)
        self._alloc_rows(f64)
        self.mean = torch.empty(p_local, **f64)
        self.sd = torch.empty(p_local, **f64)
        self.keep = torch.empty(p_local, dtype=torch.int32, device=self.dev)
        self.q = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self.G = torch.empty((self.gdim, self.gdim), **f64)
        self.ws_grm_bytes = self._grm_workspace()
        self.ws_grm = torch.empty(max(self.ws_grm_bytes, 16), dtype=torch.uint8, device=self.dev)
        self.Y = torch.zeros((nrhs, self.npad), **f64)
        self.A = torch.zeros((nrhs, self.npad), **f64)
        self.ws_solve_bytes = lib.gbm_dev_solve_workspace(n, nrhs)
        self.ws_solve = torch.empty(max(self.ws_solve_bytes, 16), dtype=torch.uint8, device=self.dev)
        # the step's host-bound results (b, GEBVs, μ̂, Σb, info) are views of one device buffer,
        # so that download() is a single D2H copy into a pinned mirror of the same layout
        shapes = [("B", (nrhs, p_local)), ("gebv", (nrhs, self.npad)), ("mu", (nrhs,)), ("msum", (nrhs,))]
        nout = sum(int(np.prod(sh)) for _, sh in shapes) + 1  # + one 8-byte slot for info
        self.out = torch.zeros(nout, **f64)
        self.h_out = torch.empty(nout, dtype=torch.float64, pin_memory=True)
        off = 0
        for name, sh in shapes:
            k = int(np.prod(sh))
            setattr(self, name, self.out[off:off + k].view(sh))
            setattr(self, "h_" + name, self.h_out[off:off + k].view(sh))
            off += k
        self.info = self.out[off:].view(torch.int32)[:1]
        self.h_info = self.h_out[off:].view(torch.int32)[:1]

    def _alloc_rows(self, f64):
        self.X = self.torch.empty((self.p, self.npad), **f64)   # raw genotypes (kept intact)
        self.Z = self.torch.empty((self.p, self.npad), **f64)   # standardised (out of place)

    def _grm_workspace(self):
        return self.lib.gbm_dev_grm_workspace(self.n, self.p)

    @staticmethod
    def _p(t):
        return ctypes.c_void_p(t.data_ptr())

    def _stream(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.dev).cuda_stream)

    def generate(self, seed: int, j0: int):
        """Synthetic genotypes for global loci j0 .. j0+p-1 (counter hash)."""
        _lib.check(self.lib.gbm_dev_synth_genotypes(self._p(self.X), self.npad, self.p, self.n, seed, j0,
                                                     self._stream()), "synth")

    def upload_genotypes(self, X_host_colmajor: np.ndarray):
        """X (n, p_local) host array → raw locus rows in HBM."""
        t = self.torch.from_numpy(np.ascontiguousarray(np.asarray(X_host_colmajor, dtype=np.float64).T))
        self.X.zero_()
        self.X[:, :self.n].copy_(t)

    def load_phenotypes(self, Y: np.ndarray):
        Y = np.asarray(Y, dtype=np.float64)
        if Y.ndim == 1:
            Y = Y[:, None]
        self.Y.zero_()
        self.Y[:, :self.n].copy_(self.torch.from_numpy(np.ascontiguousarray(Y.T)))

    # ---- stages ---------------------------------------------------------------------------
    def standardize(self):
        self.q.zero_()
        _lib.check(self.lib.gbm_dev_standardize(self._p(self.X), self.npad, self.p, self.n, self._p(self.Z), self.npad,
                                                self._p(self.mean), self._p(self.sd), self._p(self.keep),
                                                self._p(self.q), self._stream()), "standardize")

    def grm_syrk(self):
        _lib.check(self.lib.gbm_dev_grm_syrk(self._p(self.Z), self.npad, self.p, self.n, self._p(self.G), self.gdim,
                                             self._p(self.ws_grm), self.ws_grm_bytes, self._stream()), "grm_syrk")

    def grm_reduce(self):
        _lib.check(self.lib.gbm_dev_grm_reduce(self.n, self.p, self._p(self.G), self.gdim, self._p(self.ws_grm),
                                               self._stream()), "grm_reduce")

    def grm_rows(self):
        return self.G[: self.npad]

    def grm_pack(self):
        """Upper GRM tiles as one contiguous tensor, followed by q (exact as fp64: q < 2⁵³): the
        multi-GPU all-reduce operand."""
        if getattr(self, "Gp", None) is None:
            self.Gp = self.torch.empty(self.lib.gbm_dev_grm_packed_size(self.n) + 1, dtype=self.torch.float64,
                                       device=self.dev)
        _lib.check(self.lib.gbm_dev_grm_pack(self._p(self.G), self.gdim, self.n, self._p(self.Gp), self._stream()),
                   "grm_pack")
        self.Gp[-1:].copy_(self.q)
        return self.Gp

    def grm_unpack(self):
        _lib.check(self.lib.gbm_dev_grm_unpack(self._p(self.Gp), self.n, self._p(self.G), self.gdim, self._stream()),
                   "grm_unpack")
        self.q.copy_(self.Gp[-1:])

    def solve(self):
        _lib.check(self.lib.gbm_dev_gblup_solve(self._p(self.G), self.gdim, self.n, 0.0, self._p(self.q), self.lam,
                                                self._p(self.Y), self.npad, self.nrhs, self._p(self.A),
                                                self._p(self.gebv), self.npad, self._p(self.mu), self._p(self.info),
                                                self._p(self.ws_solve), self.ws_solve_bytes, self._stream()), "solve")

    # ---- the solve in phases (distributed factorisation, chol_distributed) -------------------------
    def chol_prepare(self):
        _lib.check(self.lib.gbm_dev_chol_prepare(self._p(self.G), self.gdim, self.n, 0.0, self._p(self.q), self.lam,
                                                 self._p(self.Y), self.npad, self.nrhs, self._p(self.info),
                                                 self._p(self.ws_solve), self.ws_solve_bytes, self._stream()),
                   "chol_prepare")

    def chol_prepare_cols(self, rank: int, nranks: int):
        _lib.check(self.lib.gbm_dev_chol_prepare_cols(self._p(self.G), self.gdim, self.n, 0.0, self._p(self.q),
                                                      self.lam, self._p(self.Y), self.npad, self.nrhs, rank, nranks,
                                                      self._p(self.info), self._p(self.ws_solve), self.ws_solve_bytes,
                                                      self._stream()), "chol_prepare_cols")

    def chol_group(self, kb: int, rank: int, nranks: int):
        _lib.check(self.lib.gbm_dev_chol_group(self._p(self.G), self.gdim, self.n, kb, rank, nranks, self._p(self.info),
                                               self._p(self.ws_solve), self.ws_solve_bytes, self._stream()),
                   "chol_group")

    def chol_group_panels(self, kb: int, rank: int, nranks: int):
        _lib.check(self.lib.gbm_dev_chol_group_panels(self._p(self.G), self.gdim, self.n, kb, rank, nranks,
                                                      self._p(self.info), self._p(self.ws_solve), self.ws_solve_bytes,
                                                      self._stream()), "chol_group_panels")

    def chol_group_update_cols(self, kb: int, rank: int, nranks: int, col_lo: int, col_hi: int):
        _lib.check(self.lib.gbm_dev_chol_group_update_cols(self._p(self.G), self.gdim, self.n, kb, rank, nranks, col_lo,
                                                           col_hi, self._p(self.info), self._p(self.ws_solve),
                                                           self.ws_solve_bytes, self._stream()), "chol_group_update_cols")

    def chol_group_update_tiles(self, kb: int, rank: int, nranks: int, row_lo: int, row_hi: int, col_lo: int,
                                col_hi: int):
        _lib.check(self.lib.gbm_dev_chol_group_update_tiles(self._p(self.G), self.gdim, self.n, kb, rank, nranks,
                                                            row_lo, row_hi, col_lo, col_hi, self._p(self.info),
                                                            self._p(self.ws_solve), self.ws_solve_bytes,
                                                            self._stream()), "chol_group_update_tiles")

    # the distributed solve's side stream (one per device, shared by the stages of a rehearsal; high
    # priority: the look-ahead's panels are latency-bound beside the trailing update):
    # fork = the side stream waits for this device's current stream; side() = a context in which
    # the stage methods (and a torch collective) run on it; join = the current stream waits for it
    def _side_stream(self):
        s = _SIDE_STREAMS.get(self.dev)
        if s is None:
            s = _SIDE_STREAMS[self.dev] = self.torch.cuda.Stream(self.dev, priority=-1)
        return s

    def fork(self):
        self._side_stream().wait_stream(self.torch.cuda.current_stream(self.dev))

    def side(self):
        return self.torch.cuda.stream(self._side_stream())

    def join(self):
        self.torch.cuda.current_stream(self.dev).wait_stream(self._side_stream())

    # a third stream for the deferred lower copies of the look-ahead's rows (read only by chol_finish):
    # lower_fork = it waits for the current stream; lower() = a context on it; lower_join = the current
    # stream waits for it (before chol_finish)
    def _lower_stream(self):
        s = _LOWER_STREAMS.get(self.dev)
        if s is None:
            s = _LOWER_STREAMS[self.dev] = self.torch.cuda.Stream(self.dev)
        return s

    def lower_fork(self):
        self._lower_stream().wait_stream(self.torch.cuda.current_stream(self.dev))

    def lower(self):
        return self.torch.cuda.stream(self._lower_stream())

    def lower_join(self):
        self.torch.cuda.current_stream(self.dev).wait_stream(self._lower_stream())

    def chol_lower_copy(self, kb: int, rows64: int, rank: int, nranks: int):
        _lib.check(self.lib.gbm_dev_chol_lower_copy(self._p(self.G), self.gdim, self.n, kb, rows64, rank, nranks,
                                                    self._stream()), "chol_lower_copy")

    def chol_group_update(self, kb: int, rank: int, nranks: int):
        _lib.check(self.lib.gbm_dev_chol_group_update(self._p(self.G), self.gdim, self.n, kb, rank, nranks,
                                                      self._p(self.info), self._p(self.ws_solve), self.ws_solve_bytes,
                                                      self._stream()), "chol_group_update")

    def area_pack(self, kb: int, rows64: int, rank: int, nranks: int):
        cnt = int(self.lib.gbm_dev_chol_area_doubles(self.n, kb, rows64, nranks))
        buf = self.torch.empty(max(cnt, 1), dtype=self.torch.float64, device=self.dev)[:cnt]
        _lib.check(self.lib.gbm_dev_chol_area_pack(self._p(self.G), self.gdim, self.n, kb, rows64, rank, nranks,
                                                   self._p(buf), self._stream()), "area_pack")
        return buf

    def area_unpack(self, kb: int, rows64: int, nranks: int, gathered):
        _lib.check(self.lib.gbm_dev_chol_area_unpack(self._p(self.G), self.gdim, self.n, kb, rows64, nranks,
                                                     self._p(gathered), self._stream()), "area_unpack")

    def strip_unpack_rows(self, kb: int, rows64: int, rank: int, nranks: int, gathered):
        _lib.check(self.lib.gbm_dev_chol_strip_unpack_rows(self._p(self.G), self.gdim, self.n, kb, rows64, rank, nranks,
                                                           self._p(gathered), self._stream()), "strip_unpack_rows")

    def chol_factor_diag(self, kb: int):
        _lib.check(self.lib.gbm_dev_chol_factor_diag(self._p(self.G), self.gdim, self.n, kb, self._p(self.info),
                                                     self._p(self.ws_solve), self.ws_solve_bytes, self._stream()),
                   "chol_factor_diag")

    def strip_pack(self, kb: int, rows64: int, rank: int, nranks: int):
        size = self.lib.gbm_dev_chol_strip_doubles(self.n, kb, rows64, nranks)
        buf = self.torch.empty(max(size, 2), dtype=self.torch.float64, device=self.dev)[:size]
        _lib.check(self.lib.gbm_dev_chol_strip_pack(self._p(self.G), self.gdim, self.n, kb, rows64, rank, nranks,
                                                    self._p(buf), self._stream()), "strip_pack")
        return buf

    def strip_unpack(self, kb: int, rows64: int, nranks: int, gathered):
        _lib.check(self.lib.gbm_dev_chol_strip_unpack(self._p(self.G), self.gdim, self.n, kb, rows64, nranks,
                                                      self._p(gathered), self._stream()), "strip_unpack")

    def chol_finish(self):
        _lib.check(self.lib.gbm_dev_chol_finish(self._p(self.G), self.gdim, self.n, self._p(self.Y), self.npad,
                                                self.nrhs, self.lam, self._p(self.A), self._p(self.gebv), self.npad,
                                                self._p(self.mu), self._p(self.info), self._p(self.ws_solve),
                                                self.ws_solve_bytes, self._stream()), "chol_finish")

    def effects(self):
        _lib.check(self.lib.gbm_dev_marker_effects(self._p(self.Z), self.npad, self.p, self.n, self._p(self.A),
                                                   self.npad, self.nrhs, 0.0, self._p(self.q), self._p(self.mean),
                                                   self._p(self.sd), self._p(self.keep), self._p(self.B), self.p,
                                                   self._p(self.msum), self._stream()), "effects")

    def download(self):
        self.h_out.copy_(self.out, non_blocking=True)
        self.torch.cuda.current_stream(self.dev).synchronize()
        if int(self.h_info[0]) < 0:
            raise _lib.GBMError("solve: a wait between workgroups timed out (dataflow Cholesky or back substitution; the result is invalid)")
        if int(self.h_info[0]) != 0:
            raise _lib.GBMError(f"G/q + λI not positive definite (pivot {int(self.h_info[0])})")
        return dict(B=self.h_B.numpy(), y_pred=self.h_gebv.numpy()[:, : self.n].T, mu=self.h_mu.numpy(),
                    msum=self.h_msum.numpy())


def chunk_schedule(p: int, chunk: int, halve_tail: bool = False):
    """Loci chunks [(j, pc), ...] of a streamed shard: chunks of ``chunk`` loci; with ``halve_tail`` the
    last full piece cut into halving pieces (none below 512 loci). Mirrors csrc/capi.cpp chunk_schedule
    (the C ABI halves only for copy-bound fp64 uploads at n <= 8192 or when GBM_HOST_CHUNK is set)."""
    cs, j = [], 0
    while p - j > chunk:
        cs.append((j, chunk))
        j += chunk
    r = p - j
    d = 0
    while halve_tail and d < 3 and r // 2 >= 512:
        h = r // 2
        cs.append((j, r - h))
        j += r - h
        r = h
        d += 1
    if r > 0:
        cs.append((j, r))
    return cs


class HipStreamedShardStages(HipShardStages):
    """A shard whose fp64 locus rows do not fit HBM (config C3 on one MI355X: 600 000 loci × 50 048 × 8 B
    = 240 GB beside a 20 GB G): the genotypes stay resident as int8 dosages (1 B per cell, 30 GB), and
    the loci pass through one fp64 chunk buffer — each chunk standardised from the bytes and its GRM
    added into G in place (chunk GRMs summed in chunk order); the marker effects re-read the bytes with
    z rebuilt in registers. The same chunks and kernels as the C ABI's loci-streamed mode
    (csrc/capi.cpp stream_grm_shard / stream_effects_shard), so the results are the same bits."""

    def __init__(self, n: int, p_local: int, chunk: int, nrhs: int = 1, lambda_: float = 1.0, device: int = 0,
                 ploidy: int = 2, halve_tail: bool = False):
        self.chunk = int(min(chunk, p_local))
        self.ploidy = int(ploidy)
        self.sched = chunk_schedule(p_local, self.chunk, halve_tail)
        super().__init__(n, p_local, nrhs=nrhs, lambda_=lambda_, device=device)

    def _alloc_rows(self, f64):
        self.X = None
        self.D = self.torch.empty((self.p, self.n), dtype=self.torch.int8, device=self.dev)  # Julia (n, p) layout
        self.Z = self.torch.empty((self.chunk, self.npad), **f64)  # one chunk of standardised rows

    def _grm_workspace(self):
        return max(self.lib.gbm_dev_grm_workspace(self.n, pc) for _, pc in self.sched)

    def generate(self, seed: int, j0: int):
        """Synthetic dosages (counter hash) of global loci j0 .. j0+p-1: X = D/2."""
        _lib.check(self.lib.gbm_dev_synth_dosage_i8(self._p(self.D), self.n, self.p, self.n, seed, j0, self._stream()),
                   "synth_dosage_i8")
        self.ploidy = 2

    def upload_dosages(self, D_host_colmajor: np.ndarray, ploidy: int):
        """Dosages D (n, p_local) int8 host array → resident bytes (X = D/ploidy)."""
        self.D.copy_(self.torch.from_numpy(np.ascontiguousarray(np.asarray(D_host_colmajor, dtype=np.int8).T)))
        self.ploidy = int(ploidy)

    def upload_genotypes(self, X_host_colmajor: np.ndarray):
        raise _lib.ArgumentError("a streamed shard holds int8 dosages: use upload_dosages")

    # ---- stages: standardisation runs per chunk inside grm_syrk ------------------------------------
    def standardize(self):
        self.q.zero_()

    def grm_syrk(self):
        lib, Zp, Gp, s = self.lib, self._p(self.Z), self._p(self.G), self._stream()
        for k, (j, pc) in enumerate(self.sched):
            _lib.check(lib.gbm_dev_standardize_i8(ctypes.c_void_p(self.D.data_ptr() + j * self.n), self.n, pc, self.n,
                                                  self.ploidy, Zp, self.npad, self._p(self.mean[j:]),
                                                  self._p(self.sd[j:]), self._p(self.keep[j:]), self._p(self.q), s),
                       "standardize_i8")
            if k > 0 and lib.gbm_dev_grm_slices(self.n, pc) > 1:
                _lib.check(lib.gbm_dev_grm_accumulate(Zp, self.npad, pc, self.n, Gp, self.gdim, self._p(self.ws_grm),
                                                      self.ws_grm_bytes, s), "grm_accumulate")
            elif k == 0:
                _lib.check(lib.gbm_dev_grm(Zp, self.npad, pc, self.n, Gp, self.gdim, self._p(self.ws_grm),
                                           self.ws_grm_bytes, s), "grm")
            else:  # a single-range chunk: its own G, then added (the C ABI's Gc path)
                Gc = self.torch.empty_like(self.G)
                _lib.check(lib.gbm_dev_grm(Zp, self.npad, pc, self.n, self._p(Gc), self.gdim, self._p(self.ws_grm),
                                           self.ws_grm_bytes, s), "grm")
                self.G.add_(Gc)
                del Gc

    def grm_reduce(self):
        pass

    def effects(self):
        _lib.check(self.lib.gbm_dev_marker_effects_i8(self._p(self.D), self.n, self.p, self.n, self.ploidy,
                                                      self._p(self.A), self.npad, self.nrhs, 0.0, self._p(self.q),
                                                      self._p(self.mean), self._p(self.sd), self._p(self.keep),
                                                      self._p(self.B), self.p, self._p(self.msum), self._stream()),
                   "effects_i8")

    def genotype_chunks(self):
        """(j, X[:, j:j+pc] as (pc, n) float64 on the device) over the schedule: the streamed X for checks."""
        for j, pc in self.sched:
            yield j, self.D[j:j + pc].to(self.torch.float64) / self.ploidy


class HipExactShardStages(HipStreamedShardStages):
    """A shard of diploid dosages (int8, 1 B per cell, resident) whose GRM is computed EXACTLY by the int8
    matrix cores (csrc/grm_exact.hip): G = Σ_j w_j (d_j − t_j/n)(d_j − t_j/n)ᵀ with each
    locus weight w_j = 1/var_j held as an exact fixed-point integer in base-128 digits, the digit GEMMs summed
    in int32 and the centring in int128, one rounding to fp64 at the end. No fp64 Z is ever formed; the
    marker effects re-read the bytes (as the loci-streamed shard does)."""

    def __init__(self, n: int, p_local: int, nrhs: int = 1, lambda_: float = 1.0, device: int = 0):
        self.slices = ctypes.c_int32(0)
        super().__init__(n, p_local, p_local, nrhs=nrhs, lambda_=lambda_, device=device, ploidy=2)

    def _alloc_rows(self, f64):
        self.X = None
        self.Z = None
        self.D = self.torch.empty((self.p, self.n), dtype=self.torch.int8, device=self.dev)  # Julia (n, p) layout

    def _grm_workspace(self):
        return self.lib.gbm_dev_grm_exact_workspace(self.n, self.p)

    def grm_syrk(self):
        _lib.check(self.lib.gbm_dev_grm_exact_i8(self._p(self.D), self.n, self.p, self.n, self.ploidy, self._p(self.G),
                                                 self.gdim, self._p(self.mean), self._p(self.sd), self._p(self.keep),
                                                 self._p(self.q), 0, self._p(self.ws_grm), self.ws_grm_bytes,
                                                 ctypes.byref(self.slices), self._stream()), "grm_exact_i8")

    def download(self):
        # the exact GRM's own status (a weight outside its digits' range: G invalid) before the results are used;
        # the stream is drained here anyway
        _lib.check(self.lib.gbm_dev_grm_exact_status(self._p(self.ws_grm), self.n, self.p, self._stream()),
                   "grm_exact_status")
        return super().download()
