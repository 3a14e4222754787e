"""bench.py runs its C3 CPU extrapolation (OpenBLAS over 50 000-row matrices) in a spawned child, so that a
crash there cannot take the GPU measurement's JSON line with it."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_isolated_leg_returns_result():
    assert bench.run_isolated(str, 5, timeout_s=60) == "5"


def test_isolated_leg_survives_a_crash():
    bench._CRASHES.clear()
    out = bench.run_isolated(ctypes.string_at, 0, timeout_s=60)  # SIGSEGV in the child
    assert "error" in out and "exit code" in out["error"]
    assert out["crash"]["signal"] == "SIGSEGV" and out["crash"]["exit_code"] < 0
    assert bench._CRASHES and bench._CRASHES[-1]["leg"] == "string_at"  # the line marks the run failed
    bench._CRASHES.clear()
