"""Per-kernel totals of the LAST solve in a kernel trace of tools/dist_solve_time.py (tools/dist_trace.sh), the
GPU-busy time against the solve's span, and the row updates' duration against their K chunk count (the j-th
row update of a panel group runs K = 64 j; a least-squares line gives the per-chunk and fixed costs).
Usage: python tools/dist_trace_stats.py gpurun_out/dist_trace/trace/run_kernel_trace.csv"""
import collections
import csv
import sys

import numpy as np


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "prepare_v_kernel" in r["Kernel_Name"]]
    last = rows[starts[-1]:]
    agg = collections.defaultdict(lambda: [0, 0.0])
    busy = 0.0
    for r in last:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        agg[r["Kernel_Name"][:70]][0] += 1
        agg[r["Kernel_Name"][:70]][1] += d
        busy += d
    t0 = int(last[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in last)
    print(f"solve span {(t1 - t0) / 1e6:.2f} ms, kernel time {busy / 1e3:.2f} ms (summed over streams)")
    for name, (calls, tot) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"{tot / 1e3:9.2f} ms {calls:6d} {tot / calls:9.1f} us  {name}")
    # row updates: consecutive syrk64_sub_kernel launches between panels, j = 1, 2, ... within a group
    js, ds = [], []
    j = 0
    for r in last:
        name = r["Kernel_Name"]
        if "syrk64_sub_kernel" in name:
            j += 1
            js.append(j)
            ds.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        elif "chol_panel_kernel" not in name:
            j = 0
    if js:
        a = np.vstack([np.ones(len(js)), js]).T
        fixed, per = np.linalg.lstsq(a, np.array(ds), rcond=None)[0]
        print(f"row updates: {len(js)} launches, duration ~ {fixed:.1f} + {per:.2f} j us (K = 64 j)")


if __name__ == "__main__":
    main(sys.argv[1])
