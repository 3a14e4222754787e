"""Timeline of the last GBLUP solve in a rocprofv3 --kernel-trace CSV: per kernel family, the
summed busy time and the summed gaps in front of its dispatches. Analysis tool only.
Usage: python tools/solve_timeline.py <run_kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last solve begins at the last prepare_v_kernel
start = max(i for i, r in enumerate(rows) if "prepare_v" in r["Kernel_Name"])
seq = rows[start:]
busy, gaps, cnt = defaultdict(float), defaultdict(float), defaultdict(int)
prev_end = None
for r in seq:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gbm::", "")[:40]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy[name] += (e - s) / 1e3
    if prev_end is not None:
        gaps[name] += max(0, s - prev_end) / 1e3
    cnt[name] += 1
    prev_end = e
total = (int(seq[-1]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1e3
print(f"solve span {total:.1f} us, {len(seq)} kernels, busy {sum(busy.values()):.1f} us, gaps {sum(gaps.values()):.1f} us")
for k in sorted(busy, key=lambda k: -busy[k]):
    print(f"  {k:40s} n={cnt[k]:4d} busy={busy[k]:8.1f} us ({busy[k]/cnt[k]:6.1f}/call) gap-before={gaps[k]:7.1f} us")
