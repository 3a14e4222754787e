#!/usr/bin/env python3
"""Time the exact-integer GRM stage (csrc/grm_exact.hip) and the whole GBLUP step on it, next to the fp64
path, on one GPU: python tools/exact_grm_time.py [n p]. Prints one JSON line per path."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genomicbreedingmodels.jl_amd"))

import torch  # noqa: E402

from gbm import synth  # noqa: E402
from gbm.sharded import HipExactShardStages, HipShardStages, LocalComm, sharded_gblup_step  # noqa: E402


def run(kind, n, p, steps=5, warmup=2):
    st = HipExactShardStages(n, p, device=0) if kind == "exact" else HipShardStages(n, p, device=0)
    st.generate(4242, 0)
    st.load_phenotypes(synth.qtl_phenotypes(4242, n, p, 1, device=0))
    torch.cuda.synchronize()
    for _ in range(warmup):
        sharded_gblup_step(st, LocalComm())
    torch.cuda.synchronize()
    marks = []
    t0 = time.perf_counter()
    for _ in range(steps):
        ev = {}

        def mark(label):
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            ev[label] = e
        sharded_gblup_step(st, LocalComm(), events=mark)
        marks.append(ev)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1000.0 / steps
    labels = ["begin", "standardize", "grm_syrk", "grm_reduce", "allreduce", "solve", "effects", "download"]
    stage = {b: sum(m[a].elapsed_time(m[b]) for m in marks) / steps for a, b in zip(labels[:-1], labels[1:])}
    out = {"path": kind, "n": n, "p": p, "ms_per_step": ms, "stage_ms": stage, "cells_per_s": n * p / ms * 1e3}
    if kind == "exact":
        S = st.slices.value
        out["slices"] = S
        out["grm_int8_tops"] = S * float(n) * (n + 1) * p / (stage["grm_syrk"] * 1e-3) / 1e12
        out["grm_fp64_equiv_tflops"] = float(n) * (n + 1) * p / (stage["grm_syrk"] * 1e-3) / 1e12
    print(json.dumps(out), flush=True)
    del st
    torch.cuda.empty_cache()


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    p = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
    for kind in (sys.argv[3:] or ["exact", "fp64"]):
        run(kind, n, p)
