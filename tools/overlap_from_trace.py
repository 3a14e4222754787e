"""Reads a rocprofv3 --kernel-trace --memory-copy-trace CSV pair of tools/two_shard_overlap.py and
reports, for the last gbm_gblup_fit call in it, how much of the host-to-device genotype copies ran
while a GRM tile kernel (syrk_kernel) was executing, and the span of the copies and of the GRM
kernels. Usage: overlap_from_trace.py <trace dir> [label]. Prints one JSON line. Timing tool only."""
import csv
import glob
import json
import sys

d = sys.argv[1]
label = sys.argv[2] if len(sys.argv) > 2 else d
kf = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
mf = glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True)[0]
kr = list(csv.DictReader(open(kf)))
mr = list(csv.DictReader(open(mf)))
col = lambda rows, *names: next((c for c in names if rows and c in rows[0]), None)
dir_col = col(mr, "Direction", "Kind", "Operation")
size_col = col(mr, "Bytes", "Size", "Copy_Bytes")
grm = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kr if "syrk_kernel<2>" in r["Kernel_Name"]
             or "syrk_kernel<1>" in r["Kernel_Name"])
grm_stream = {(int(r["Start_Timestamp"]), int(r["End_Timestamp"])): r.get("Stream_Id") for r in kr
              if "syrk_kernel" in r["Kernel_Name"]}
# the genotype chunks: pageable host memory is staged, so rocprofv3 lists those copies as
# device-to-device blits on the shard's copy stream; every copy longer than 0.25 ms is one
h2d = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r) for r in mr
             if int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) > 250_000)
if not grm or not h2d:
    print(json.dumps({"label": label, "error": "no GRM kernels or no large H2D copies", "columns": list(mr[0].keys()) if mr else []}))
    sys.exit(0)
# the last call: the GRM kernels and copies after the last gap > 5 ms between consecutive copies
starts = [c[0] for c in h2d]
cut = 0
for i in range(1, len(h2d)):
    if starts[i] - h2d[i - 1][1] > 5_000_000:
        cut = i
h2d = h2d[cut:]
t0 = h2d[0][0]
grm = [g for g in grm if g[1] >= t0]


def overlap(a0, a1):
    return sum(max(0, min(a1, g1) - max(a0, g0)) for g0, g1 in grm)


copy_ns = sum(c[1] - c[0] for c in h2d)
ov_ns = sum(overlap(c[0], c[1]) for c in h2d)
stream_col = col(mr, "Stream_Id", "Queue_Id")
streams = sorted({c[2].get(stream_col) for c in h2d}) if stream_col else []
per_stream = {}
for c in h2d:
    s = c[2].get(stream_col) if stream_col else "all"
    a = per_stream.setdefault(s, [c[0], c[1], 0, 0])
    a[0], a[1] = min(a[0], c[0]), max(a[1], c[1])
    a[2] += c[1] - c[0]
    a[3] += overlap(c[0], c[1])
print(json.dumps({
    "label": label,
    "h2d_copies": len(h2d), "h2d_busy_ms": copy_ns / 1e6, "h2d_ms_overlapping_grm": ov_ns / 1e6,
    "first_copy_to_last_grm_ms": (max(g[1] for g in grm) - t0) / 1e6,
    "grm_kernels": len(grm), "grm_first_start_ms": (grm[0][0] - t0) / 1e6,
    "per_copy_stream": {str(k): {"span_ms": [(v[0] - t0) / 1e6, (v[1] - t0) / 1e6], "busy_ms": v[2] / 1e6,
                                 "ms_overlapping_grm": v[3] / 1e6} for k, v in per_stream.items()},
    "grm_spans_ms_stream": [[(g0 - t0) / 1e6, (g1 - t0) / 1e6, grm_stream.get((g0, g1))] for g0, g1 in grm],
}))
