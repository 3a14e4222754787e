"""tools/dist_trace_stats.py (the distributed-solve kernel trace summary behind
profiles/r05_dist_solve_r8_kernel_stats.txt): only the last solve enters the totals, the span and the summed
kernel time are those of that solve, and the row-update fit recovers the per-chunk cost."""
import csv
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tool():
    spec = importlib.util.spec_from_file_location("dist_trace_stats", os.path.join(ROOT, "tools", "dist_trace_stats.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _trace(path, solves=2):
    """Each solve: prepare 40 µs, then two groups of panel / row-update launches (row update j lasts
    20 + 3 j µs), a trailing update of 100 µs on stream 0 beside a side-stream kernel of 50 µs (timestamps
    in ns, as rocprofv3 writes them)."""
    rows, t = [], 1000

    def launch(name, dur, stream=0, start=None):
        nonlocal t
        s0 = t if start is None else start
        rows.append({"Kernel_Name": name, "Start_Timestamp": str(s0), "End_Timestamp": str(s0 + 1000 * dur),
                     "Stream_Id": str(stream)})
        if start is None:
            t = s0 + 1000 * dur + 5000

    for _ in range(solves):
        launch("gbm::prepare_v_kernel(double*)", 40)
        for _g in range(2):
            launch("gbm::chol_panel_kernel(double*)", 10)
            for j in range(1, 4):
                launch("void gbm::syrk64_sub_kernel<true>(double const*)", 20 + 3 * j)
                launch("gbm::chol_panel_kernel(double*)", 10)
            s = t
            launch("void gbm::syrk_kernel<0>(double const*)", 100)
            launch("gbm::chol_group_kernel(double*)", 50, stream=1, start=s)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Stream_Id"])
        w.writeheader()
        w.writerows(rows)


def test_last_solve_totals_and_row_update_fit(tmp_path, capsys):
    p = tmp_path / "run_kernel_trace.csv"
    _trace(p)
    _tool().main(str(p))
    out = capsys.readouterr().out
    lines = {ln.split("us  ")[-1]: ln for ln in out.splitlines() if "us  " in ln}
    # the last solve only: 2 trailing updates, 6 row updates
    assert "     2 " in lines["void gbm::syrk_kernel<0>(double const*)"]
    assert "     6 " in lines["void gbm::syrk64_sub_kernel<true>(double const*)"]
    assert "duration ~ 20.0 + 3.00 j us" in out
    span = float(out.split("solve span ")[1].split(" ms")[0])
    busy = float(out.split("kernel time ")[1].split(" ms")[0])
    assert busy > span  # the side-stream kernels overlap the trailing updates
