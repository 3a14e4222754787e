"""tools/rocprof_stats.py: the warm-up-excluded per-kernel summaries committed under profiles/ (VERDICT r04 item 9).
A synthetic rocprofv3 kernel trace of a bench-like run — W warm-up + K timed steps of a path (standardise, GRM,
solve kernels), then another path reusing the solve kernels, plus one-off setup launches — is summarised; the
warm-up launches, the setup and the other path's launches must not enter the averages."""
import csv
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tool():
    spec = importlib.util.spec_from_file_location("rocprof_stats", os.path.join(ROOT, "tools", "rocprof_stats.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _trace(path, warmup, steps):
    """Kernel durations: step s of the fp64 path takes std 10+s, syrk 100 (warm-up: 150), chol 20; then the
    exact path's steps launch xg 50 and chol 30 (the shared solve kernel, slower there)."""
    rows, t = [], 1000

    def launch(name, dur):
        nonlocal t
        rows.append({"Kernel_Name": name, "Start_Timestamp": str(t), "End_Timestamp": str(t + dur)})
        t += dur + 5

    launch("synth_kernel(setup)", 7)
    for s in range(warmup + steps):
        warm = s < warmup
        launch("standardize_kernel<256>", 10 + s)
        launch("syrk_kernel<2>", 150 if warm else 100)
        launch("chol_flow_kernel<false>", 20)
    for s in range(warmup + steps):
        launch("xg_stats_kernel", 3)
        launch("xg_gemm_kernel<9>", 50)
        launch("chol_flow_kernel<false>", 30)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        w.writerows(rows)


def test_step_start_windows_exclude_warmup_setup_and_other_paths(tmp_path):
    tool = _tool()
    p = tmp_path / "run_kernel_trace.csv"
    W, K = 2, 5
    _trace(p, W, K)
    rows = {r["Name"]: r for r in tool.summarise_anchored(tool.load(str(p)), W, K, "standardize_kernel")}
    assert set(rows) == {"standardize_kernel<256>", "syrk_kernel<2>", "chol_flow_kernel<false>"}
    assert rows["syrk_kernel<2>"]["Calls"] == K and rows["syrk_kernel<2>"]["AverageNs"] == 100
    assert rows["syrk_kernel<2>"]["WarmupExcluded"] == W
    assert rows["chol_flow_kernel<false>"]["Calls"] == K and rows["chol_flow_kernel<false>"]["AverageNs"] == 20
    assert rows["standardize_kernel<256>"]["AverageNs"] == sum(10 + s for s in range(W, W + K)) / K
    exact = {r["Name"]: r for r in tool.summarise_anchored(tool.load(str(p)), W, K, "xg_stats_kernel")}
    assert set(exact) == {"xg_stats_kernel", "xg_gemm_kernel<9>", "chol_flow_kernel<false>"}
    assert exact["chol_flow_kernel<false>"]["AverageNs"] == 30 and exact["chol_flow_kernel<false>"]["Calls"] == K


def test_plain_summary_drops_the_first_warmup_launches(tmp_path):
    tool = _tool()
    p = tmp_path / "run_kernel_trace.csv"
    W, K = 1, 3
    _trace(p, W, K)
    rows = {r["Name"]: r for r in tool.summarise(tool.load(str(p)), W, K)}
    assert rows["syrk_kernel<2>"]["AverageNs"] == 100 and rows["syrk_kernel<2>"]["Calls"] == K
    assert "synth_kernel(setup)" not in rows  # one-off launches do not divide into the steps
    assert abs(sum(r["Percentage"] for r in rows.values()) - 100.0) < 1e-9
