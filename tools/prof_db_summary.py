#!/usr/bin/env python3
"""Per-kernel duration summary of a rocprofv3 SQLite result (run_results.db): name, count, average,
minimum and total microseconds, largest total first. python tools/prof_db_summary.py DB [--skip-first]"""
import collections
import sqlite3
import sys

db = sys.argv[1]
skip = "--skip-first" in sys.argv
c = sqlite3.connect(db)
agg = collections.defaultdict(list)
for name, start, end in c.execute("select name, start, end from kernels order by start"):
    agg[name].append((end - start) / 1e3)
print(f"{'kernel':70s} {'n':>4s} {'avg_us':>10s} {'min_us':>10s} {'total_us':>11s}")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    if skip and len(v) > 1:
        v = v[1:]
    print(f"{k[:70]:70s} {len(v):4d} {sum(v) / len(v):10.1f} {min(v):10.1f} {sum(v):11.1f}")
