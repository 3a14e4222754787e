"""Per-kernel statistics of a rocprofv3 --kernel-trace run with the bench's warm-up steps left out.

rocprofv3's own *_kernel_stats.csv averages every launch, the warm-up ones included (the first GRM
launch of a process is ~10 % slower). A bench run of W warm-up + K timed steps launches each per-step
kernel c = m (W + K) times; this drops the first m W launches of every such kernel (launch order) and
keeps kernels that do not divide evenly (one-off setup) out of the table.

    python tools/rocprof_stats.py <trace dir or kernel_trace.csv> --warmup W --steps K [--csv out.csv]
    python tools/rocprof_stats.py <trace> --warmup W --steps K --step-start standardize_kernel   # one path of a mixed run
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


def summarise_anchored(launches, warmup, steps, first):
    """The timed steps of one path of a run whose other paths launch some of the same kernels (bench.py: the
    fp64 stage path, then the exact-GRM path's solves, then the host path's chunked GRMs). `first` names the
    kernel that starts each step of the path (bench.py's fp64 path: standardize_kernel; the exact path:
    xg_stats_kernel), launched first in the run by that path. Step k = the launches from the k-th launch of
    `first` up to the next; the kernels of the first timed step define the step's kernel set, and the last timed
    step ends at the first later launch that is outside that set or starts another step."""
    names = sorted((min(launches[n])[0], n) for n in launches if first in n)  # the earliest-launched match
    if not names:
        sys.exit(f"step-start kernel {first!r} matches no kernel")
    names = [names[0][1]]
    f = sorted(launches[names[0]])
    if len(f) < warmup + steps or steps < 2:
        sys.exit("need warmup + steps launches of the step-start kernel and >= 2 timed steps")
    allv = sorted((s0, e0, n) for n, ls in launches.items() for s0, e0 in ls)
    start, second, last = f[warmup][0], f[warmup + 1][0], f[warmup + steps - 1][0]
    step_set = {n for s0, _, n in allv if start <= s0 < second}
    end = float("inf")
    for s0, _, n in allv:
        if s0 > last and (n not in step_set or n == names[0]):
            end = s0
            break
    kept = defaultdict(list)
    for s0, e0, n in allv:
        if start <= s0 < end:
            kept[n].append(e0 - s0)
    out, total = [], 0
    for n, d in kept.items():
        total += sum(d)
        out.append({"Name": n, "Calls": len(d), "WarmupExcluded": len(launches[n]) - len(d), "TotalNs": sum(d),
                    "AverageNs": sum(d) / len(d), "MinNs": min(d), "MaxNs": max(d)})
    for r in out:
        r["Percentage"] = 100.0 * r["TotalNs"] / total if total else 0.0
    return sorted(out, key=lambda r: -r["TotalNs"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--step-start", help="kernel name part launched first in each step of the path to summarise "
                                         "(bench.py's fp64 stage path: standardize_kernel; exact path: xg_stats_kernel)")
    ap.add_argument("--csv")
    a = ap.parse_args()
    if a.step_start:
        rows = summarise_anchored(load(a.trace), a.warmup, a.steps, a.step_start)
    else:
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
