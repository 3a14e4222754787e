"""Per-kernel statistics of a rocprofv3 --kernel-trace run with the bench's warm-up steps left out.

rocprofv3's own *_kernel_stats.csv averages every launch, the warm-up ones included (the first GRM
launch of a process is ~10 % slower). A bench run of W warm-up + K timed steps launches each per-step
kernel c = m (W + K) times; this drops the first m W launches of every such kernel (launch order) and
keeps kernels that do not divide evenly (one-off setup) out of the table.

    python tools/rocprof_stats.py <trace dir or kernel_trace.csv> --warmup W --steps K [--csv out.csv]
"""
import argparse
import csv
import glob
import os
import sys
from collections import defaultdict


def load(path):
    if os.path.isdir(path):
        files = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        if not files:
            sys.exit(f"no *kernel_trace.csv under {path}")
        path = files[0]
    rows = list(csv.DictReader(open(path)))
    launches = defaultdict(list)
    for r in rows:
        launches[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return launches


def summarise(launches, warmup, steps):
    out, total = [], 0
    for name, ls in launches.items():
        ls.sort()
        per = len(ls) / float(warmup + steps)
        if per != int(per) or per == 0:
            continue
        kept = ls[int(per) * warmup:]
        d = [e - s for s, e in kept]
        total += sum(d)
        out.append({"Name": name, "Calls": len(d), "WarmupExcluded": len(ls) - len(d), "TotalNs": sum(d),
                    "AverageNs": sum(d) / len(d), "MinNs": min(d), "MaxNs": max(d)})
    for r in out:
        r["Percentage"] = 100.0 * r["TotalNs"] / total if total else 0.0
    return sorted(out, key=lambda r: -r["TotalNs"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--csv")
    a = ap.parse_args()
    rows = summarise(load(a.trace), a.warmup, a.steps)
    cols = ["Name", "Calls", "WarmupExcluded", "TotalNs", "AverageNs", "MinNs", "MaxNs", "Percentage"]
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=cols)
            w.writeheader()
            w.writerows(rows)
    for r in rows[:15]:
        print(f"{r['Name'][:60]:60s} {r['Calls']:5d} {r['AverageNs'] / 1000:10.1f} us {r['Percentage']:6.2f} %")


if __name__ == "__main__":
    main()
