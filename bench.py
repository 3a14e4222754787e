#!/usr/bin/env python3
"""GRM + GBLUP benchmark (BASELINE.json metric: genotype-cells/s = n·p / wall time).

Workload (config C2 of BASELINE.json, per GPU): GBLUP on n = 5 000 individuals × p = 50 000 loci,
fp64, λ = 1, one trait. Genotypes are generated on the device by the counter-based hash of
SURVEY.md §8d (bit-identical to the oracle's generator), so they are resident in HBM before the
timed region. With N ranks (torchrun, one process per GPU) each rank owns a different block of
50 000 loci (weak scaling over loci: p_total = 50 000·N); the partial GRMs are summed by an RCCL
all-reduce over xGMI.

A step = standardise → fp64-MFMA GRM → (all-reduce) → Cholesky GBLUP solve → marker effects →
results (b, GEBVs, μ̂) copied to pinned host memory.

`--stream-chunk C` runs the loci-streamed mode instead (config C3 on one GPU: `--individuals 50000
--loci 600000 --stream-chunk 75000`): the genotypes resident as int8 dosages (1 B per cell), each
chunk of C loci standardised and added into G in place, the marker effects from the bytes.

The C3 leg (`--c3-leg`, on by default whenever N > 1): after the headline, every rank
runs BASELINE.json configs[2] — n = 50 000, 600 000 loci SPLIT over the N ranks (75 000 per rank at N = 8, int8
dosages resident, 75 000-locus fp64 chunks), the packed RCCL all-reduce of the partial GRMs, the distributed
Cholesky (strip all-gathers) — 1 warm-up + 2 timed steps, reported under the line's "c3" key with the GRM and
end-to-end fractions of N x the fp64 peak and every rank's GRM / all-reduce / solve / all-gather-wait times. The
N = 1 headline is unchanged.

Parity (rank 0, N = 1, when the oracle can run the same problem): the numpy restatement fits the
SAME genotypes and phenotypes the GPU step fitted; the line carries rel_err of y_pred, μ̂, b_hat and
q equality.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))

PEAK_F64_TFLOPS = 78.6  # MI355X fp64 matrix peak (AMD datasheet)
PEAK_HBM_GBS = 8000.0
PEAK_I8_TOPS = 5000.0  # MI355X dense int8 MFMA (2x bf16 per clock: MI355X_MICROARCH.md, Matrix cores)
# back-to-back v_mfma_i32_16x16x64_i8 with the exact GEMM's 36 accumulators and one v_perm per MFMA, all CUs,
# random operands (tools/mfma_i8_rate.hip, profiles/r04_mfma_i8_rate.jsonl; 3.8-4.7 POPS without the perms)
MEASURED_I8_LOOP_TOPS = 3620.0
MEASURED_MFMA_F64_TFLOPS = 74.1  # back-to-back v_mfma_f64_16x16x4_f64 loop, tools/mfma_f64_probe.hip


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one process per GPU). N > 1 without torchrun's WORLD_SIZE: this process starts "
                         "torch.distributed.run with N ranks as a child and relays its line")
    ap.add_argument("--collectives", choices=("auto", "always"), default="auto",
                    help="always: run the step's collectives (packed partial-GRM all-reduce, Cholesky strip "
                         "all-gathers from n >= GBM_DIST_SOLVE_MIN_N) even at world size 1, over a 1-rank "
                         "process group of --dist-backend (RCCL by default)")
    ap.add_argument("--launch-check", action="store_true",
                    help="harness check without GPU work: rendezvous, barriers, max-over-ranks timing and the "
                         "rank-0 line around an empty step (value null); for CPU tests of the N-rank launcher")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--individuals", type=int, default=5000)
    ap.add_argument("--loci", type=int, default=50000, help="loci per GPU")
    ap.add_argument("--nrhs", type=int, default=1)
    ap.add_argument("--lam", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=4242)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cpu-c3", action="store_true", help="skip the extrapolated C3 CPU baseline")
    ap.add_argument("--no-host-path", action="store_true", help="skip the C-ABI (host buffer) timings")
    ap.add_argument("--cpu-sample-p", type=int, default=0, help="loci in the CPU baseline sample (0 = all)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL); gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--same-device", action="store_true", help="all ranks on cuda:0 (rehearsal on a 1-GPU box)")
    ap.add_argument("--stream-chunk", type=int, default=0,
                    help="loci per chunk of the loci-streamed mode (int8 dosages resident); 0 = resident fp64 X")
    ap.add_argument("--no-exact", action="store_true", help="skip the exact-integer GRM measurement beside the fp64 line")
    ap.add_argument("--c3-leg", choices=("auto", "on", "off"), default="auto",
                    help="the C3 leg (BASELINE.json configs[2], the north star): after the headline, n = --c3-individuals "
                         "x --c3-loci loci SPLIT over the launched ranks (strong scaling), loci-streamed fp64 GRM, "
                         "packed RCCL all-reduce, distributed Cholesky; auto = on when more than one rank runs")
    ap.add_argument("--c3-individuals", type=int, default=50000)
    ap.add_argument("--c3-loci", type=int, default=600000, help="loci in total (split over the ranks)")
    ap.add_argument("--c3-chunk", type=int, default=75000, help="loci per fp64 chunk of a rank's streamed shard")
    ap.add_argument("--c3-steps", type=int, default=2)
    ap.add_argument("--c3-warmup", type=int, default=1)
    ap.add_argument("--c3-seed", type=int, default=424242)
    ap.add_argument("--c3-timeout", type=float, default=300.0, help="watchdog of the C3 leg (seconds)")
    ap.add_argument("--c3-exact", choices=("auto", "on", "off"), default="auto",
                    help="also time C3 with the exact-integer GRM (the drop-in default on diploid data) after the fp64 "
                         "leg; auto = whenever the C3 leg runs")
    ap.add_argument("--grm", choices=("fp64", "exact"), default="fp64",
                    help="fp64: the fp64-MFMA SYRK on standardised rows; exact: int8 dosages resident, the GRM "
                         "computed exactly by int8-MFMA digit GEMMs with int128 centring (csrc/grm_exact.hip)")
    return ap.parse_args()


# BASELINE.json configs this bench can run (n, loci in total); the line names the one it ran
CONFIGS = {(5000, 50000): "C2 GBLUP 5 000 x 50 000 (BASELINE.json configs[1])",
           (50000, 600000): "C3 GBLUP 50 000 x 600 000 (BASELINE.json configs[2])",
           (50000, 75000): "C3's per-GPU shard 50 000 x 75 000 (1/8 of BASELINE.json configs[2])"}


def workload_label(n, p_local, world, stream_chunk, exact=False):
    """config.workload from (n, p, N): weak scaling keeps p_local loci per GPU, so the per-GPU shape
    names the config (C2: 5 000 x 50 000 per GPU), and a one-GPU run over all loci of C3 names C3."""
    p_total = p_local * world
    name = CONFIGS.get((n, p_local)) if world > 1 else CONFIGS.get((n, p_total))
    name = name or f"custom GBLUP n={n} x p={p_total} (no BASELINE.json config)"
    mode = (f"loci-streamed ({stream_chunk}-locus fp64 chunks, int8 dosages resident)" if stream_chunk
            else "int8 dosages resident, exact-integer GRM" if exact else "fp64 X resident")
    return (f"{name}: n={n} x p={p_local} loci per GPU, p_total={p_total} over {world} GPU(s), {mode}"
            + (", loci-sharded, partial GRMs all-reduced" if world > 1 else ""))


def _blas_threads():
    try:
        from threadpoolctl import threadpool_info
        return max([d.get("num_threads", 1) for d in threadpool_info() if d.get("internal_api") == "openblas"] or [1])
    except Exception:  # pragma: no cover
        return len(os.sched_getaffinity(0))


def _oracle_c():
    """The C/OpenMP restatement (oracle/gbm_oracle.c, built by build()), or None."""
    import ctypes
    so = os.path.join(ROOT, "oracle", "build", "libgbm_oracle.so")
    if not os.path.exists(so):
        return None
    lib = ctypes.CDLL(so)
    V, I = ctypes.c_void_p, ctypes.c_int64
    lib.gbm_ref_synth_matrix.argtypes = [ctypes.c_uint64, I, I, I, V, I]
    lib.gbm_ref_gblup_fit.restype = I
    lib.gbm_ref_gblup_fit.argtypes = [V, I, I, I, V, I, I, ctypes.c_double, V, V, V, V]
    return lib


def cpu_baseline(args, Y, gpu):
    """The CPU restatements of the hot path on the same workload (rank 0, N = 1), each one full
    GBLUP fit (standardise + GRM + Cholesky + solves + marker effects) on n x p_sample with the
    genotypes generated beforehand (untimed): the numpy/OpenBLAS restatement (oracle/oracle.py,
    the headline `value`) and the plain C/OpenMP restatement (oracle/gbm_oracle.c). Both are this
    build's ports of the reference's equations (the Julia reference cannot run here: SURVEY §0.7).

    The fit uses the phenotypes Y of the GPU step, so with the full sample (p_sample = p) it is the
    same problem the GPU solved: returns (baseline, parity) with parity = rel_err of y_pred, μ̂,
    b_hat against the GPU step's results and q equality."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    threads = _blas_threads()
    n = args.individuals
    p = args.cpu_sample_p or args.loci
    lib = _oracle_c()
    X = np.zeros((n, p), order="F")
    if lib is not None:
        lib.gbm_ref_synth_matrix(args.seed, n, p, 0, X.ctypes.data, n)
    else:
        X = O.synth_genotypes(args.seed, n, p)
    Y = np.asfortranarray(Y)
    t0 = time.perf_counter()
    ref = O.gblup_fit(X, Y, args.lam)
    dt = time.perf_counter() - t0
    out = {"value": n * p / dt, "unit": "genotype-cells/s", "cores": int(threads), "kind": "port",
           "sample": f"numpy/OpenBLAS fp64 restatement (oracle/oracle.py gblup_fit) on n={n} x p={p}, "
                     f"{args.nrhs} trait(s), one full fit in {dt:.2f} s (standardise + GRM + Cholesky + solves + "
                     f"marker effects; generation untimed)"}
    if p == args.loci:
        parity = parity_of(gpu, ref)
        parity.update({"n": n, "p": p})
    else:
        parity = {"skipped": f"CPU sample p={p} differs from the GPU step's p={args.loci}"}
        ref = None
    if lib is not None:
        t = args.nrhs
        b = np.zeros((p + 1, t), order="F")
        yp = np.zeros((n, t), order="F")
        mu = np.zeros(t)
        q = np.zeros(1, dtype=np.int64)
        omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
        t0 = time.perf_counter()
        rc = lib.gbm_ref_gblup_fit(X.ctypes.data, n, p, n, Y.ctypes.data, n, t, args.lam, b.ctypes.data,
                                   yp.ctypes.data, mu.ctypes.data, q.ctypes.data)
        dtc = time.perf_counter() - t0
        assert rc == 0 and np.abs(yp - ref["y_pred"]).max() < 1e-8 * np.abs(ref["y_pred"]).max()
        out["c_openmp"] = {"value": n * p / dtc, "unit": "genotype-cells/s", "cores": omp, "kind": "port",
                           "sample": f"plain C/OpenMP restatement (oracle/gbm_oracle.c gbm_ref_gblup_fit, gcc -O3 "
                                     f"-fopenmp) on the same n={n} x p={p} fit: {dtc:.2f} s; GEBVs equal the numpy "
                                     f"fit's to 1e-8"}
    return out, parity, ref


def parity_of(gpu, ref):
    """rel. errors of y_pred, μ̂, b_hat of a GPU fit against the oracle's fit of the same X and Y."""
    def rel(a, b):
        return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(np.abs(np.asarray(b)).max(), 1e-300))
    parity = {"oracle": "oracle/oracle.py gblup_fit (numpy/LAPACK fp64) on the same X and Y as the GPU step",
              "q_equal": int(ref["q"]) == int(gpu["q"]),
              "rel_err_y_pred": rel(gpu["y_pred"], ref["y_pred"]), "rel_err_mu": rel(gpu["mu"], ref["mu"]),
              "rel_err_b_hat": rel(gpu["b_hat"], ref["b_hat"]), "tolerance_y_pred": 1e-9}
    parity["pass"] = bool(parity["q_equal"] and parity["rel_err_y_pred"] < 1e-9 and parity["rel_err_mu"] < 1e-9
                          and parity["rel_err_b_hat"] < 1e-6)
    return parity


def cpu_baseline_c3(args):
    """CPU time of config C3 (GBLUP n = 50 000 x p = 600 000), extrapolated: the full problem (240 GB
    of fp64 X, 1.5e15 GRM flops) cannot run on the host in a bench. The numpy/OpenBLAS restatement's
    per-fit costs are timed on samples and combined: standardise + GRM + marker effects at
    n = 50 000 on p = 10 000 and 20 000 loci (linear in p: slope = cost per locus, intercept = the
    n x n output), and the Cholesky + solves at n = 16 000 scaled by (50 000/16 000)^3. BASELINE.md
    planned p = 60 000 and 120 000; those samples take ~10 min of CPU each, beyond a bench run, so
    the line uses the largest samples that keep this leg near half a minute."""
    import scipy.linalg as sla
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    lib = _oracle_c()
    n, p3 = 50000, 600000

    def gen(n, p):
        X = np.zeros((n, p), order="F")
        if lib is not None:
            lib.gbm_ref_synth_matrix(424242, n, p, 0, X.ctypes.data, n)
        else:
            X = O.synth_genotypes(424242, n, p)
        return X

    def grm_effects(X):
        # the unique triangle by dsyrk (numpy's own Z @ Z.T takes OpenBLAS's syrk path, which
        # crashes at a 50 000 x 50 000 output on this image)
        a = np.random.default_rng(1).standard_normal(X.shape[0])
        t0 = time.perf_counter()
        m, s, keep = O.colstats(X)
        Z = np.asfortranarray(O.standardize(X, m, s, keep))
        G = sla.blas.dsyrk(1.0 / Z.shape[1], Z)
        (Z.T @ a) / Z.shape[1]
        dt = time.perf_counter() - t0
        del G, Z
        return dt

    samples = {}
    pa, pb = 10000, 20000
    for p in (pa, pb):
        X = gen(n, p)
        samples[p] = grm_effects(X)
        del X
    slope = (samples[pb] - samples[pa]) / float(pb - pa)
    icpt = samples[pa] - pa * slope
    nc = 16000
    rng = np.random.default_rng(2)
    Xc = gen(nc, 2000)
    m, s, keep = O.colstats(Xc)
    Z = np.asfortranarray(O.standardize(Xc, m, s, keep))
    V = sla.blas.dsyrk(1.0 / Z.shape[1], Z)
    V[np.diag_indices(nc)] += 1.0
    del Z, Xc
    rhs = np.column_stack([np.ones(nc), rng.standard_normal(nc)])
    t0 = time.perf_counter()
    c = sla.cho_factor(V, lower=False, overwrite_a=True, check_finite=False)  # dsyrk filled the upper triangle
    sla.cho_solve(c, rhs, check_finite=False)
    t_chol = time.perf_counter() - t0
    del V, c
    t_chol_c3 = t_chol * (n / nc) ** 3
    t_c3 = slope * p3 + icpt + t_chol_c3
    return {"value": n * p3 / t_c3, "unit": "genotype-cells/s", "cores": int(_blas_threads()), "kind": "port",
            "extrapolated": True, "seconds_c3": t_c3,
            "sample": f"EXTRAPOLATION of the numpy/OpenBLAS restatement to C3 (n=50000 x p=600000): standardise + "
                      f"GRM + marker effects timed at n=50000 on p={pa} ({samples[pa]:.2f} s) and p={pb} "
                      f"({samples[pb]:.2f} s), linear in p -> {slope * p3 + icpt:.1f} s at p=600000; Cholesky + "
                      f"solves timed at n=16000 ({t_chol:.2f} s) x (50000/16000)^3 -> {t_chol_c3:.1f} s; "
                      f"total {t_c3:.1f} s on one host"}


def _cpu_baseline_packed(packed):
    """cpu_baseline(*packed) for the isolated child; the oracle fit comes back without its n x n arrays."""
    out, parity, ref = cpu_baseline(*packed)
    if ref is not None:
        ref = {k: ref[k] for k in ("q", "y_pred", "mu", "b_hat")}
    return out, parity, ref


def _isolated_child(fn, args, conn):
    import faulthandler
    faulthandler.enable()  # a fatal signal in the leg prints every thread's Python stack to stderr
    try:
        conn.send(("ok", fn(args)))
    except Exception as e:  # pragma: no cover - reported by the parent
        conn.send(("error", repr(e)))
    conn.close()


def run_isolated(fn, args, timeout_s=400):
    """fn(args) in a fresh interpreter (spawn: no torch, no HIP): the C3 CPU extrapolation drives OpenBLAS
    dsyrk/potrf over 50 000-row matrices, and a crash there must not take the GPU measurement with it.
    Returns fn's result, or {"error": ...} when the child fails, crashes or times out."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    parent, child = ctx.Pipe(duplex=False)
    p = ctx.Process(target=_isolated_child, args=(fn, args, child))
    p.start()
    child.close()
    out = {"error": f"the isolated CPU leg did not answer within {timeout_s} s"}
    if parent.poll(timeout_s):
        try:
            status, val = parent.recv()
            out = val if status == "ok" else {"error": val}
        except EOFError:
            pass
    p.join(10)
    if p.is_alive():
        p.kill()
        p.join()
    if p.exitcode not in (0, None):
        import signal
        crash = {"exit_code": p.exitcode,
                 "signal": signal.Signals(-p.exitcode).name if p.exitcode < 0 else None,
                 "leg": getattr(fn, "__name__", str(fn))}
        if isinstance(out, dict) and "error" in out:
            out["error"] += f" (child exit code {p.exitcode})"
            out["crash"] = crash
        _CRASHES.append(crash)
    return out


_CRASHES = []  # isolated CPU legs that died (exit code / signal): reported in the line, the run marked failed


def host_path(args, torch):
    """The product entry a Julia ccall binds (gbm_gblup_fit, X handed over in host memory), on the
    same workload (rank 0, N = 1): pageable and pinned X, the int8-dosage entry, and the H2D copy
    of X alone. PCIe-inclusive, so never the bench `value` (which starts with X in HBM)."""
    import ctypes

    import gbm
    from gbm import _lib, synth

    n, p, t = args.individuals, args.loci, args.nrhs
    lib = gbm.load_library()
    Xd = synth.genotypes_device(args.seed, n, p)  # (p, npad) locus rows
    Y = np.asfortranarray(synth.qtl_phenotypes(args.seed, n, p, t))
    pinned = torch.empty((p, n), dtype=torch.float64, pin_memory=True)
    pinned.copy_(Xd[:, :n])
    X_pin = pinned.numpy().T  # (n, p) column-major view of pinned memory
    X_page = np.asfortranarray(X_pin.copy())
    D_page = np.asfortranarray(np.rint(X_page * 2.0).astype(np.int8))
    del Xd
    torch.cuda.empty_cache()
    b = np.zeros((p + 1, t), order="F")
    yp = np.zeros((n, t), order="F")
    mu = np.zeros(t)
    q = np.zeros(1, dtype=np.int64)

    def fit_f64(X):
        _lib.check(lib.gbm_gblup_fit(_lib.ptr(X), n, p, n, _lib.ptr(Y), n, t, args.lam, None, 0, _lib.ptr(b),
                                     _lib.ptr(yp), _lib.ptr(mu), _lib.ptr(q)), "gbm_gblup_fit")

    def fit_auto(X):  # the drop-in's mode on dosage-valued X: the device dosage check + the exact GRM
        used = ctypes.c_int(-1)
        _lib.check(lib.gbm_gblup_fit_ex(_lib.ptr(X), n, p, n, _lib.ptr(Y), n, t, args.lam, None, 0, _lib.GBM_GRM_AUTO,
                                        _lib.ptr(b), _lib.ptr(yp), _lib.ptr(mu), _lib.ptr(q), ctypes.byref(used)),
                   "gbm_gblup_fit_ex(auto)")
        assert used.value == _lib.GBM_GRM_EXACT

    def fit_i8():
        _lib.check(lib.gbm_gblup_fit_dosage_i8(_lib.ptr(D_page), n, p, n, 2, _lib.ptr(Y), n, t, args.lam, None, 0,
                                               _lib.ptr(b), _lib.ptr(yp), _lib.ptr(mu), _lib.ptr(q)),
                   "gbm_gblup_fit_dosage_i8")

    def timed(fn, reps=3):
        fn()  # warm-up: pooled context allocated
        a0 = lib.gbm_device_allocations()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        dt = (time.perf_counter() - t0) / reps
        assert lib.gbm_device_allocations() == a0
        return dt * 1000.0

    ms_page = timed(lambda: fit_f64(X_page))
    ms_pin = timed(lambda: fit_f64(X_pin))
    ms_i8 = timed(fit_i8)
    ms_auto = timed(lambda: fit_auto(X_page))
    ms_auto_pin = timed(lambda: fit_auto(X_pin))
    dev_buf = torch.empty((p, n), dtype=torch.float64, device="cuda")

    def h2d(src):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            dev_buf.copy_(src)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / 3 * 1000.0

    h2d_pin = h2d(pinned)
    h2d_page = h2d(torch.from_numpy(np.ascontiguousarray(X_page.T)))
    del dev_buf
    return {
        "entry": "gbm_gblup_fit (C ABI, host X column-major n x p; Julia ccall path) on the same workload",
        "ms_per_call_pageable_x": ms_page, "ms_per_call_pinned_x": ms_pin, "ms_per_call_dosage_i8": ms_i8,
        "ms_per_call_auto_f64_x": ms_auto, "ms_per_call_auto_f64_x_pinned": ms_auto_pin,
        "auto_note": "gbm_gblup_fit_ex(GBM_GRM_AUTO) on the same pageable (and pinned) fp64 X: the drop-in gblup's "
                     "default on diploid data (julia/gblup.jl grm = :dropin with GBM_GRM unset) — 2x checked and packed "
                     "to dosage bytes on the host by up to 16 threads (GBM_HOST_PACK=1, the default), 1 B per cell over "
                     "PCIe chunk by chunk, then the exact-integer GRM (DESIGN.md §4.8)",
        "host_pack": {"enabled": os.environ.get("GBM_HOST_PACK", "1") != "0",
                      "threads": int(os.environ.get("GBM_PACK_THREADS", "0") or 0) or min(16, len(os.sched_getaffinity(0)))},
        "h2d_x_ms_pinned": h2d_pin, "h2d_x_ms_pageable": h2d_page, "x_bytes": 8 * n * p,
        "cells_per_s_pinned_x": n * p / (ms_pin / 1000.0), "device_allocations_per_call_after_warmup": 0,
    }


def load_pmc(n, p):
    """HBM traffic per GRM launch from the committed rocprofv3 PMC summary, if one matches the shape.
    Returns (bytes or None, stale): stale when the GRM kernel source has changed since the counters
    were taken (the summary records the sha256 of csrc/grm.hip; tools/pmc_summary.py)."""
    import hashlib
    path = os.path.join(ROOT, "profiles", "pmc_grm.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    if d.get("n") != n or d.get("p") != p:
        return None, None
    with open(os.path.join(ROOT, "genomicbreedingmodels.jl_amd", "csrc", "grm.hip"), "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()
    return d.get("hbm_bytes_per_launch"), d.get("grm_hip_sha256") != sha


class TimedComm:
    """A comm (TorchComm) whose collectives are bracketed by timing events on the stream that issues them (the
    compute stream, or the distributed solve's side stream): per collective kind, the time that stream spent from
    issuing the collective to its completion (waiting for the slowest rank included)."""

    def __init__(self, comm, torch):
        self.comm, self.torch = comm, torch
        self.world_size, self.rank = comm.world_size, comm.rank
        self.force = getattr(comm, "force", False)
        self.spans = []  # (kind, bytes, event before, event after)

    def _timed(self, kind, fn, t):
        e0 = self.torch.cuda.Event(enable_timing=True)
        e1 = self.torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn(t)
        e1.record()
        self.spans.append((kind, int(t.numel() * t.element_size()), e0, e1))
        return out

    def all_reduce_sum(self, t):
        return self._timed("all_reduce", self.comm.all_reduce_sum, t)

    def all_gather(self, t):
        return self._timed("all_gather", self.comm.all_gather, t)

    def take(self):
        """{kind: [ms, calls, bytes]} of the spans recorded since the last take (events complete: call after a
        synchronize)."""
        out = {}
        for kind, nb, e0, e1 in self.spans:
            acc = out.setdefault(kind, [0.0, 0, 0])
            acc[0] += e0.elapsed_time(e1)
            acc[1] += 1
            acc[2] += nb
        self.spans = []
        return out


def c3_split(p_total, world, rank):
    """(j0, p_local) of rank's contiguous block of loci: ceil(p/world) per rank."""
    per = (p_total + world - 1) // world
    j0 = min(rank * per, p_total)
    return j0, max(0, min(per, p_total - j0))


def c3_record(n, p_total, world, steps, warmup, ms_per_step, per_rank, chunk, backend, slices=None):
    """rank 0's `c3` object from the leg's timings: per_rank = one dict per rank with its mean per-step stage
    times (grm = standardise + GRM of its loci, allreduce, solve, effects) and collective spans. The fractions
    count the algorithmic flops of SURVEY.md §8d (GRM n(n+1)p, Cholesky n³/3, solves 8n², back-solve 2np) against
    N x the fp64 MFMA peak."""
    grm_flops = float(n) * (n + 1) * p_total
    chol_flops = float(n) ** 3 / 3.0
    other = 8.0 * float(n) ** 2 + 2.0 * n * p_total
    grm_ms = max((r.get("grm_ms") or 0.0) for r in per_rank) if per_rank else 0.0
    peak = world * PEAK_F64_TFLOPS * 1e12
    ok = ms_per_step is not None and ms_per_step > 0
    if slices:  # the exact-integer GRM: S int8 digit GEMMs of n(n+1)p ops against N x the int8 peak
        ops = slices * grm_flops
        return {
            "workload": f"C3 GBLUP {n} x {p_total} with the exact-integer GRM (the drop-in default on diploid data): "
                        f"the loci split over {world} rank(s), int8 dosages resident, {slices} int8-MFMA digit GEMMs + "
                        f"int128 centring per rank, packed partial-GRM all-reduce ({backend}), distributed Cholesky; "
                        f"strong scaling",
            "n": n, "p_total": p_total, "ranks": world, "steps": steps, "warmup": warmup, "ms_per_step": ms_per_step,
            "value": n * p_total / (ms_per_step / 1000.0) if ok else None, "unit": "genotype-cells/s",
            "digit_slices": slices,
            "grm_int8_frac_of_peak": ops / (grm_ms / 1000.0) / (world * PEAK_I8_TOPS * 1e12) if grm_ms > 0 else None,
            "grm_ms_max_over_ranks": grm_ms, "peak_tops_per_gpu": PEAK_I8_TOPS, "backend": backend,
            "per_rank": per_rank,
        }
    return {
        "workload": f"C3 GBLUP {n} x {p_total} (BASELINE.json configs[2] at n=50000, p=600000): the loci split over "
                    f"{world} rank(s) ({-(-p_total // world)} per rank, int8 dosages resident, {chunk}-locus fp64 "
                    f"chunks), packed partial-GRM all-reduce ({backend}), distributed Cholesky; strong scaling",
        "n": n, "p_total": p_total, "ranks": world, "steps": steps, "warmup": warmup,
        "ms_per_step": ms_per_step,
        "value": n * p_total / (ms_per_step / 1000.0) if ok else None, "unit": "genotype-cells/s",
        "grm_frac_of_peak": grm_flops / (grm_ms / 1000.0) / peak if grm_ms > 0 else None,
        "grm_ms_max_over_ranks": grm_ms,
        "e2e_fp64_frac_of_peak": (grm_flops + chol_flops + other) / (ms_per_step / 1000.0) / peak if ok else None,
        "peak_tflops_per_gpu": PEAK_F64_TFLOPS, "backend": backend,
        "per_rank": per_rank,
    }


def run_c3_leg(args, torch, dist, base_comm, world, rank, dev, exact=False):
    """The C3 leg: n x p_total over the launched ranks, each rank a contiguous block of loci
    (int8 dosages generated in HBM, standardised per fp64 chunk into the partial GRM), the packed all-reduce of the
    upper tiles + q, the distributed Cholesky from n >= GBM_DIST_SOLVE_MIN_N (each rank its own tile columns,
    strip all-gathers), marker effects; W untimed + K timed steps between barrier + synchronize pairs, max over
    ranks. Every rank returns its record; rank 0's carries every rank's stage times."""
    import gbm
    from gbm import synth
    from gbm.sharded import HipExactShardStages, HipStreamedShardStages, sharded_gblup_step

    n, p_total = args.c3_individuals, args.c3_loci
    j0, p_local = c3_split(p_total, world, rank)
    chunk = min(args.c3_chunk, p_local)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    gbm.load_library().gbm_release_device_cache()
    if exact:
        st = HipExactShardStages(n, p_local, nrhs=1, lambda_=args.lam, device=dev)
    else:
        st = HipStreamedShardStages(n, p_local, chunk, nrhs=1, lambda_=args.lam, device=dev)
    st.generate(args.c3_seed, j0)
    Y = synth.qtl_phenotypes(args.c3_seed, n, p_total, 1, device=dev)
    st.load_phenotypes(Y)
    comm = TimedComm(base_comm, torch)
    labels = ["begin", "standardize", "grm_syrk", "grm_reduce", "allreduce", "solve", "effects", "download"]
    for _ in range(args.c3_warmup):
        sharded_gblup_step(st, comm)
    torch.cuda.synchronize()
    comm.take()
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    recs, out = [], None
    t0 = time.perf_counter()
    for _ in range(args.c3_steps):
        evs = {}

        def mark(label, evs=evs):
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            evs[label] = e
        out = sharded_gblup_step(st, comm, events=mark)
        recs.append(evs)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist.is_initialized():
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    K = max(args.c3_steps, 1)
    stage = {}
    for a, b in zip(labels[:-1], labels[1:]):
        stage[b] = float(np.mean([r[a].elapsed_time(r[b]) for r in recs]))
    coll = comm.take()
    y = np.asarray(out["y_pred"])
    mine = {"rank": rank, "loci": p_local, "j0": j0,
            "grm_ms": stage["standardize"] + stage["grm_syrk"] + stage["grm_reduce"],
            "allreduce_ms": stage["allreduce"], "solve_ms": stage["solve"], "effects_ms": stage["effects"],
            "download_ms": stage["download"],
            "allgather_blocked_ms": coll.get("all_gather", [0.0])[0] / K,
            "allgather_calls": coll.get("all_gather", [0, 0])[1] // K,
            "allgather_bytes_received": coll.get("all_gather", [0, 0, 0])[2] * world // K,
            "allreduce_span_ms": coll.get("all_reduce", [0.0])[0] / K,
            "allreduce_bytes": coll.get("all_reduce", [0, 0, 0])[2] // K,
            "q": int(st.q.item()), "y_pred_finite": bool(np.all(np.isfinite(y))),
            "y_pred_sum": float(y.sum()), "mu": float(out["mu"][0])}
    per_rank = [mine]
    if dist.is_initialized():
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    slices = int(st.slices.value) if exact else None
    del st
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    backend = dist.get_backend() if dist.is_initialized() else "none"
    rec = c3_record(n, p_total, world, args.c3_steps, args.c3_warmup, elapsed * 1000.0 / K, per_rank, chunk,
                    "RCCL" if backend == "nccl" else backend, slices=slices)
    # every rank solved the same summed system: identical GEBVs (the distributed factorisation is bit-identical to
    # the redundant one); q = p_total (MAF >= 0.05: every locus polymorphic at this n)
    rec["ranks_agree"] = len({(r["y_pred_sum"], r["mu"]) for r in per_rank}) == 1
    rec["q"] = per_rank[0]["q"]
    return rec


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv):
    """`bench.py --gpus N` (N > 1) run without torchrun: start `python -m torch.distributed.run
    --nproc-per-node N ... bench.py <same arguments>` as a CHILD process (one rank per GPU; this parent
    never touches the GPU: torch.cuda.device_count() does not initialise HIP) and exit with its code. The
    ranks' rank-0 line goes straight to this process's stdout. Refuses (exit 3) when fewer than N devices
    are visible, unless --same-device (all ranks on cuda:0: a rehearsal) or --launch-check."""
    import subprocess
    n = args.gpus
    if not (args.same_device or args.launch_check):
        import torch
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py: --gpus {n} needs {n} visible GPUs, found {have}; refusing to time fewer ranks "
                  f"than asked (use --same-device to rehearse {n} ranks on one GPU)", file=sys.stderr, flush=True)
            return 3
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # RCCL over dmabuf IPC only on this pool
    return subprocess.call(cmd, env=env)


def init_ranks(args, torch, dist):
    """(world, rank, device index) of this process; initialises the process group for N > 1 ranks (and for
    --collectives always at one rank, a 1-rank group)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were launched")
    dev_idx = 0 if (args.same_device or world == 1) else local_rank
    if not args.launch_check:
        torch.cuda.set_device(dev_idx)
    if world > 1 or args.collectives == "always":
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if args.dist_backend == "nccl" and not args.launch_check:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx))
        else:
            dist.init_process_group("gloo" if args.launch_check else args.dist_backend)
        world = dist.get_world_size()
        rank = dist.get_rank()
    return world, rank, dev_idx


def launch_check(args, torch, dist, world, rank):
    """The N-rank harness around an empty step (no GPU): barrier, K timed steps, max over ranks, one line."""
    def sync():
        if world > 1 or dist.is_initialized():
            dist.barrier()
    for _ in range(args.warmup):
        pass
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    sync()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if dist.is_initialized():
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        ranks = [None] * world
        dist.all_gather_object(ranks, {"rank": rank, "pid": os.getpid()})
    else:
        ranks = [{"rank": 0, "pid": os.getpid()}]
    c3 = None
    if args.c3_leg == "on" or (args.c3_leg == "auto" and world > 1):  # the record's shape around empty timings
        pr = [{"rank": r, "loci": c3_split(args.c3_loci, world, r)[1], "j0": c3_split(args.c3_loci, world, r)[0],
               "grm_ms": 0.0, "allreduce_ms": 0.0, "solve_ms": 0.0, "effects_ms": 0.0, "download_ms": 0.0,
               "allgather_blocked_ms": 0.0, "allgather_calls": 0, "allgather_bytes_received": 0,
               "allreduce_span_ms": 0.0, "allreduce_bytes": 0} for r in range(world)]
        c3 = c3_record(args.c3_individuals, args.c3_loci, world, args.c3_steps, args.c3_warmup, None, pr,
                       min(args.c3_chunk, pr[0]["loci"]), dist.get_backend() if dist.is_initialized() else "none")
        if args.c3_exact != "off":
            c3["exact_grm_leg"] = sorted(c3_record(args.c3_individuals, args.c3_loci, world, args.c3_steps,
                                                   args.c3_warmup, None, pr, 0, "none", slices=9))
    if rank == 0:
        print(json.dumps({"metric": "GRM+GBLUP genotype-cells/s (n x p)", "value": None, "unit": "genotype-cells/s", "c3": c3,
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": float(el.item()) * 1000.0 / max(args.steps, 1), "higher_is_better": True,
                          "scaling": "weak", "launch_check": True,
                          "note": "harness check only (--launch-check): empty step, no GPU work, not a measurement",
                          "world_size": world, "backend": dist.get_backend() if dist.is_initialized() else None,
                          "ranks": ranks}), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def headline_record(args, n, p_local, p_total, world, value, ms_per_step, syrk_ms, stage_ms, per_rank, exact,
                    grm_slices, digit_slices, dist):
    """rank 0's line (the headline step) before the C3 leg and the host/CPU legs add to it."""
    # algorithmic work of SURVEY.md §8d: GRM n(n+1)p (unique triangle of the rank-p update),
    # Cholesky n³/3, solves 8n² per right-hand side (four triangular solves), back-solve 2np
    grm_flops = float(n) * (n + 1) * p_local
    chol_flops = float(n) ** 3 / 3.0
    solve_flops = 8.0 * float(n) ** 2 * args.nrhs + 2.0 * n * p_local * args.nrhs
    achieved = grm_flops / (syrk_ms / 1000.0) / 1e12
    traffic, traffic_stale = load_pmc(n, p_local) if not (args.stream_chunk or exact) else (None, None)
    e2e_frac = (grm_flops + chol_flops + solve_flops) / (ms_per_step / 1000.0) / (PEAK_F64_TFLOPS * 1e12)

    rec = {
        "metric": "GRM+GBLUP genotype-cells/s (n x p)",
        "value": value,
        "unit": "genotype-cells/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("i8 digit GEMMs (exact int32 sums) + int128 centring -> f64 G; f64 solve" if exact else "f64"),
        "data": "synthetic: counter-hash genotypes (MAF U(0.05,0.5), dosage Binomial(2,f), X=d/2) generated in HBM"
                + (" as int8 dosages" if (args.stream_chunk or exact) else " as fp64") + "; 1% QTL phenotype, h2=0.5",
        "config": {
            "workload": workload_label(n, p_local, world, args.stream_chunk, exact),
            "n": n, "p_per_gpu": p_local, "p_total": p_total, "traits": args.nrhs, "lambda": args.lam,
            "grm_slices": grm_slices,
            "grm_digit_slices": digit_slices,
            "stream_chunk": args.stream_chunk or None,
            "parallelism": f"loci-shard x{world}",
        },
        "roofline": {
            "bound": "mfma",
            "kernel": "GRM stage: syrk_kernel<kPersist> (fp64 v_mfma_f64_16x16x4_f64 128x128 tiles) + "
                      "grm_edge_kernel (ragged last column); achieved = all n(n+1)p flops / stage time"
                      + ("; streamed: the stage also standardises each chunk from the int8 dosages"
                         if args.stream_chunk else ""),
            "achieved": achieved,
            "peak": PEAK_F64_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved / PEAK_F64_TFLOPS,
            "frac_of_measured_mfma": achieved / MEASURED_MFMA_F64_TFLOPS,
            "measured_mfma_peak": MEASURED_MFMA_F64_TFLOPS,
            "traffic": traffic,
            "traffic_source": "profiles/pmc_grm.json: rocprofv3 --pmc FETCH_SIZE (x2, gfx950 16 B/lane "
                              "under-count) + WRITE_SIZE per GRM launch, separate passes of this command"
                              if traffic is not None else None,
            "traffic_stale": traffic_stale,
            "flops_per_launch": grm_flops,
            "ms_per_launch": syrk_ms,
        },
        "stage_ms": stage_ms,
        "e2e_fp64_frac_of_peak": e2e_frac,
        "world_size": world,
        "backend": dist.get_backend() if dist.is_initialized() else None,
        "collectives": ("RCCL" if dist.is_initialized() and dist.get_backend() == "nccl" else
                        dist.get_backend() if dist.is_initialized() else "none (one rank)")
                       + (" (forced at one rank: --collectives always)" if world == 1 and dist.is_initialized() else ""),
        "per_rank_stage_ms": per_rank if world > 1 or dist.is_initialized() else None,
    }
    if exact:
        S = digit_slices
        ops = S * grm_flops  # S digit GEMMs of n(n+1)/2 x p int8 multiply-adds (2 ops each)
        tops = ops / (syrk_ms / 1000.0) / 1e12
        rec["roofline"] = {
            "bound": "mfma",
            "kernel": f"GRM stage: xg_gemm_kernel<{S}> (v_mfma_i32_16x16x64_i8, {S} base-128 digit GEMMs of the fixed-"
                      "point locus weights, 128x64 upper tiles) + its per-locus prep kernels (stats, digits, transpose, "
                      "int128 centring terms); achieved = S n(n+1)p int8 ops / stage time",
            "achieved": tops, "peak": PEAK_I8_TOPS, "unit": "TOPS (int8)", "frac": tops / PEAK_I8_TOPS,
            "frac_of_measured_i8_loop": tops / MEASURED_I8_LOOP_TOPS, "measured_i8_loop": MEASURED_I8_LOOP_TOPS,
            "traffic": None, "ops_per_launch": ops, "ms_per_launch": syrk_ms,
        }
        rec["e2e_fp64_frac_of_peak"] = None
    return rec


def c3_watchdog(args, rank, rec):
    """A daemon timer: after --c3-timeout seconds rank 0 prints its line with "c3" = an error (the headline is
    complete) and every rank leaves with os._exit(0), so a hung collective cannot cost the whole run's line."""
    import threading

    def fire():
        if rank == 0:
            key = "c3_exact_grm" if "c3" in rec else "c3"  # (a finished fp64 leg keeps its record)
            rec[key] = {"error": f"the C3 leg did not finish within {args.c3_timeout} s (watchdog); the headline "
                                 f"fields of this line are complete"}
            print(json.dumps(rec), flush=True)
        sys.stderr.write(f"bench.py rank {rank}: C3 leg watchdog fired after {args.c3_timeout} s\n")
        sys.stderr.flush()
        os._exit(0)
    t = threading.Timer(args.c3_timeout, fire)
    t.daemon = True
    t.start()
    return t


def main():
    import faulthandler
    faulthandler.enable()
    args = parse()
    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    import torch
    import torch.distributed as dist

    world, rank, dev_idx = init_ranks(args, torch, dist)
    if args.launch_check:
        return launch_check(args, torch, dist, world, rank)
    dev = torch.cuda.current_device()

    import gbm
    from gbm import synth
    from gbm.sharded import (HipExactShardStages, HipShardStages, HipStreamedShardStages, LocalComm, TorchComm,
                             assemble_b_hat, sharded_gblup_step)

    comm = TorchComm(force=args.collectives == "always") if dist.is_initialized() else LocalComm()
    n, p_local = args.individuals, args.loci
    p_total = p_local * world
    j0 = rank * p_local
    exact = args.grm == "exact"
    if exact:
        st = HipExactShardStages(n, p_local, nrhs=args.nrhs, lambda_=args.lam, device=dev)
    elif args.stream_chunk:
        st = HipStreamedShardStages(n, p_local, args.stream_chunk, nrhs=args.nrhs, lambda_=args.lam, device=dev)
    else:
        st = HipShardStages(n, p_local, nrhs=args.nrhs, lambda_=args.lam, device=dev)
    st.generate(args.seed, j0)
    Y = synth.qtl_phenotypes(args.seed, n, p_total, args.nrhs, device=dev)
    st.load_phenotypes(Y)
    torch.cuda.synchronize()

    labels = ["begin", "standardize", "grm_syrk", "grm_reduce", "allreduce", "solve", "effects", "download"]

    def run_steps(st):
        """W untimed steps, then K steps timed between barrier + synchronize pairs (max over ranks);
        returns (ms per step, mean per-stage event times, the last step's results)."""
        recs = []

        def make_marks():
            evs = {}

            def mark(label):
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                evs[label] = e
            return evs, mark

        for _ in range(args.warmup):
            sharded_gblup_step(st, comm)
        torch.cuda.synchronize()
        if dist.is_initialized():
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = None
        for _ in range(args.steps):
            evs, mark = make_marks()
            out = sharded_gblup_step(st, comm, events=mark)
            recs.append(evs)
        torch.cuda.synchronize()
        if dist.is_initialized():
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        if dist.is_initialized():
            t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        stage = {}
        for a, b in zip(labels[:-1], labels[1:]):
            stage[b] = float(np.mean([r[a].elapsed_time(r[b]) for r in recs]))
        return elapsed * 1000.0 / args.steps, stage, out

    ms_per_step, stage_ms, out = run_steps(st)
    syrk_ms = stage_ms["grm_syrk"]
    per_rank = [stage_ms]
    if dist.is_initialized():  # every rank's own stage times (GRM, all-reduce, solve ...), on rank 0
        per_rank = [None] * world
        dist.all_gather_object(per_rank, stage_ms)
    value = n * p_total / (ms_per_step / 1000.0)

    # the exact-integer GRM path (§4.8) on the same genotypes and phenotypes, measured beside the fp64
    # headline at N = 1: int8 dosages resident, the GRM exact up to each locus weight's fp64 rounding
    alt = None
    if world == 1 and not exact and not args.stream_chunk and not args.no_exact:
        q_fp64 = int(st.q.item())
        ex = HipExactShardStages(n, p_local, nrhs=args.nrhs, lambda_=args.lam, device=dev)
        ex.generate(args.seed, j0)
        ex.load_phenotypes(Y)
        torch.cuda.synchronize()
        ems, estage, eout = run_steps(ex)
        S = int(ex.slices.value)
        grm_ops = S * float(n) * (n + 1) * p_local
        tops = grm_ops / (estage["grm_syrk"] / 1000.0) / 1e12
        alt = {"path": "exact-integer GRM (bench.py --grm exact; csrc/grm_exact.hip, DESIGN.md §4.8): int8 dosages "
                       "resident, G = exact int8-MFMA digit GEMMs + int128 centring, one fp64 rounding; f64 solve",
               "value": n * p_total / (ems / 1000.0), "unit": "genotype-cells/s", "ms_per_step": ems,
               "speedup_vs_fp64_path": ms_per_step / ems, "stage_ms": estage, "digit_slices": S,
               "q_equal_fp64_path": int(ex.q.item()) == q_fp64,
               "roofline": {"bound": "mfma", "kernel": f"xg_gemm_kernel<{S}> + prep kernels (GRM stage)",
                            "achieved": tops, "peak": PEAK_I8_TOPS, "unit": "TOPS (int8)", "frac": tops / PEAK_I8_TOPS,
                            "frac_of_measured_i8_loop": tops / MEASURED_I8_LOOP_TOPS,
                            "measured_i8_loop": MEASURED_I8_LOOP_TOPS, "ops_per_launch": grm_ops},
               "gpu": {"y_pred": eout["y_pred"], "mu": eout["mu"], "q": int(ex.q.item()),
                       "b_hat": assemble_b_hat(eout["mu"], eout["msum"], [eout["B"]], p_local)}}
        del ex
        torch.cuda.empty_cache()

    # sanity: finite GEBVs, b0 assembled
    assert np.all(np.isfinite(out["y_pred"])) and np.all(np.isfinite(out["B"]))

    head_q = int(st.q.item())
    grm_slices = int(st.lib.gbm_dev_grm_slices(n, args.stream_chunk or p_local)) if not exact else None
    digit_slices = int(st.slices.value) if exact else None
    rec = headline_record(args, n, p_local, p_total, world, value, ms_per_step, syrk_ms, stage_ms, per_rank, exact,
                          grm_slices, digit_slices, dist) if rank == 0 else None

    # the C3 leg (north star, BASELINE.json configs[2]): on by default whenever more than one rank runs. A watchdog
    # bounds it: should a collective hang, rank 0 prints the headline line (its "c3" an error) and every rank exits
    if args.c3_leg == "on" or (args.c3_leg == "auto" and world > 1):
        del st  # the headline shard's HBM back before the C3 shard is allocated
        dog = c3_watchdog(args, rank, rec)

        def leg(exact):
            try:
                return run_c3_leg(args, torch, dist, comm, world, rank, dev, exact=exact)
            except Exception as e:  # a failed leg is reported in the line; the headline stands
                import traceback
                traceback.print_exc()
                err = {"error": f"the C3 leg ({'exact' if exact else 'fp64'} GRM) failed: {e!r}"}
                if world > 1:  # the other ranks may be inside a collective: end the run after the line
                    if rank == 0:
                        rec["c3_exact_grm" if exact else "c3"] = err
                        print(json.dumps(rec), flush=True)
                    os._exit(0)
                return err
        c3 = leg(False)
        if rank == 0:
            rec["c3"] = c3
        if args.c3_exact != "off":
            c3x = leg(True)
            if rank == 0:
                rec["c3_exact_grm"] = c3x
        dog.cancel()

    if rank != 0:
        dist.destroy_process_group()
        return
    if world == 1 and not args.no_host_path and not args.stream_chunk and float(n) * p_local <= 2e9:
        rec["host_path"] = host_path(args, torch)
        rec["stage_ms"]["h2d_x_pinned"] = rec["host_path"]["h2d_x_ms_pinned"]
    oracle_fits = float(n) * p_local <= 5e8 and args.cpu_sample_p in (0, p_local)  # ~seconds on the host
    if world == 1 and not args.no_cpu_baseline and oracle_fits:
        gpu = {"y_pred": out["y_pred"], "mu": out["mu"], "q": head_q,
               "b_hat": assemble_b_hat(out["mu"], out["msum"], [out["B"]], p_local)}
        res = run_isolated(_cpu_baseline_packed, (args, np.asarray(Y), gpu))
        if isinstance(res, dict):  # the child failed: no baseline, no parity from this run
            rec["cpu_baseline"], rec["parity"], ref = res, {"skipped": "CPU leg failed: " + res["error"]}, None
        else:
            rec["cpu_baseline"], rec["parity"], ref = res
        if alt is not None and ref is not None:
            alt["parity"] = parity_of(alt["gpu"], ref)
        if not args.no_cpu_c3:
            rec["cpu_baseline_c3_extrapolated"] = run_isolated(cpu_baseline_c3, args)
    elif world == 1 and not args.no_cpu_baseline and (n, p_local) == (50000, 600000):
        rec["cpu_baseline"] = run_isolated(cpu_baseline_c3, args)  # C3: the full fit cannot run on the host
        rec["parity"] = {"skipped": "the oracle cannot fit 50 000 x 600 000 on the host; C3 is checked by "
                                    "tests/test_gpu_large.py::test_c3_full_size_one_gpu_streamed (exact-solution "
                                    "properties, C ABI vs stage path)"}
    else:
        rec["cpu_baseline"] = None
        rec["parity"] = {"skipped": "multi-rank run, or --no-cpu-baseline, or a size the oracle cannot fit in seconds"}
    if alt is not None:
        alt.pop("gpu", None)
        rec["exact_grm_path"] = alt
    if _CRASHES:  # a CPU leg died: a finding, not a footnote (its stack is on stderr via faulthandler)
        rec["run_ok"] = False
        rec["cpu_leg_crashes"] = _CRASHES
    print(json.dumps(rec), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
