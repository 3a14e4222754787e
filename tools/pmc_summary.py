"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes for the
GRM SYRK kernel (gfx950 correction: FETCH_SIZE counts half the bytes of 16-B/lane streaming
reads, MI355X_MICROARCH.md §HBM — doubled here; WRITE_SIZE taken as is; both in KiB)."""
import csv
import glob
import json
import os
import sys


def per_kernel(path_glob, counter):
    vals = {}
    for f in glob.glob(path_glob, recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r.get("Kernel_Name", "")
            vals.setdefault(name, []).append(float(r["Counter_Value"]))
    return vals


def main(root):
    fetch = per_kernel(os.path.join(root, "FETCH_SIZE", "**", "*counter_collection*.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(root, "WRITE_SIZE", "**", "*counter_collection*.csv"), "WRITE_SIZE")
    bench = json.load(open(os.path.join(root, "bench_FETCH_SIZE.json")))
    import hashlib
    src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "genomicbreedingmodels.jl_amd", "csrc", "grm.hip")
    out = {"n": bench["config"]["n"], "p": bench["config"]["p_per_gpu"], "kernels": {},
           # bench.py flags roofline.traffic stale once the GRM kernel source differs from this
           "grm_hip_sha256": hashlib.sha256(open(src, "rb").read()).hexdigest()}
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, [])
        w = write.get(name, [])
        fk = sum(f) / len(f) if f else None
        wk = sum(w) / len(w) if w else None
        out["kernels"][name[:120]] = {
            "launches": max(len(f), len(w)),
            "fetch_kib_raw": fk, "write_kib": wk,
            "hbm_bytes_per_launch": ((2 * fk if fk else 0) + (wk or 0)) * 1024 if (fk or wk) else None,
        }
    # the GRM stage = syrk_kernel<2> (kPersist; <1> = kSplit when persistence is off) + the
    # ragged-column grm_edge_kernel; syrk_kernel<0> is the Cholesky trailing update
    syrk = [v for k, v in out["kernels"].items() if "syrk_kernel<2>" in k or "syrk_kernel<1>" in k]
    edge = [v for k, v in out["kernels"].items() if "grm_edge_kernel" in k]
    if syrk:
        out["syrk_bytes_per_launch"] = syrk[0]["hbm_bytes_per_launch"]
        out["edge_bytes_per_launch"] = edge[0]["hbm_bytes_per_launch"] if edge else 0
        out["hbm_bytes_per_launch"] = (syrk[0]["hbm_bytes_per_launch"] or 0) + (out["edge_bytes_per_launch"] or 0)
        out["algorithmic_bytes_per_launch"] = 8.0 * out["n"] * out["p"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
