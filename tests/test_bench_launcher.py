"""bench.py's N-rank launcher on CPU: `bench.py --gpus N` without torchrun's WORLD_SIZE
starts `torch.distributed.run --nproc-per-node N` as a child and relays its rank-0 line; it refuses (exit 3)
when fewer than N GPUs are visible; a --gpus that disagrees with the launched WORLD_SIZE is an error. The
rendezvous, barriers, max-over-ranks timing and the line are checked around an empty step (--launch-check:
no GPU work, value null), over gloo with 127.0.0.1 as the master address."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env=None, timeout=180):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout, env=e,
                          cwd=ROOT)


def test_gpus_2_launches_two_ranks_and_prints_one_line():
    out = _run(["--gpus", "2", "--dist-backend", "gloo", "--same-device", "--launch-check", "--steps", "3",
                "--warmup", "1"])
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["world_size"] == 2 and rec["backend"] == "gloo"
    assert rec["launch_check"] is True and rec["value"] is None
    ranks = rec["ranks"]
    assert [r["rank"] for r in ranks] == [0, 1] and len({r["pid"] for r in ranks}) == 2
    assert all(r["pid"] != os.getpid() for r in ranks)


def test_gpus_4_launch_check():
    out = _run(["--gpus", "4", "--same-device", "--launch-check", "--steps", "2", "--warmup", "0"])
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["n_gpus"] == 4 and len(rec["ranks"]) == 4


def test_refuses_more_gpus_than_visible():
    """On a box with fewer GPUs than asked (none here) the bench exits non-zero with a message instead of
    timing fewer ranks."""
    out = _run(["--gpus", "8", "--steps", "1", "--warmup", "0"], env={"HIP_VISIBLE_DEVICES": ""})
    assert out.returncode == 3
    assert "needs 8 visible GPUs" in out.stderr
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]


def test_gpus_must_match_launched_world_size():
    env = {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}
    out = _run(["--gpus", "2", "--launch-check"], env=env)
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr


def test_c3_leg_record_at_two_ranks():
    """--gpus 2 turns the C3 leg on (auto): the line carries the "c3" record with the loci split over the two
    ranks, the fractions' fields and one stage-time entry per rank (timings empty under --launch-check)."""
    out = _run(["--gpus", "2", "--same-device", "--launch-check", "--steps", "1", "--warmup", "0"])
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
    c3 = rec["c3"]
    assert c3["n"] == 50000 and c3["p_total"] == 600000 and c3["ranks"] == 2
    assert [r["loci"] for r in c3["per_rank"]] == [300000, 300000]
    assert [r["j0"] for r in c3["per_rank"]] == [0, 300000]
    for key in ("ms_per_step", "value", "grm_frac_of_peak", "e2e_fp64_frac_of_peak", "steps", "warmup", "workload"):
        assert key in c3
    for key in ("grm_ms", "allreduce_ms", "solve_ms", "allgather_blocked_ms", "allgather_calls"):
        assert all(key in r for r in c3["per_rank"])
    assert "strong scaling" in c3["workload"]
    # the exact-integer GRM leg that follows (its record's keys; launch-check has no timings)
    assert {"digit_slices", "grm_int8_frac_of_peak", "per_rank", "value"} <= set(c3["exact_grm_leg"])


def test_c3_leg_off_at_one_rank_by_default():
    out = _run(["--launch-check", "--steps", "1", "--warmup", "0"])
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["c3"] is None


def test_c3_record_arithmetic():
    """bench.c3_record: value = n p / time; GRM fraction from the slowest rank's GRM stage over N x peak; e2e from
    all algorithmic flops."""
    sys.path.insert(0, ROOT)
    import bench
    pr = [{"grm_ms": 2000.0}, {"grm_ms": 2500.0}]
    r = bench.c3_record(50000, 600000, 8, 2, 1, 3000.0, pr, 75000, "RCCL")
    rx = bench.c3_record(50000, 600000, 8, 2, 1, 800.0, pr, 0, "RCCL", slices=9)
    assert abs(rx["grm_int8_frac_of_peak"] - 9 * 50000.0 * 50001 * 600000 / 2.5 / (8 * 5000e12)) < 1e-12
    assert abs(r["value"] - 50000 * 600000 / 3.0) < 1e-3
    grm = 50000.0 * 50001 * 600000
    assert abs(r["grm_frac_of_peak"] - grm / 2.5 / (8 * 78.6e12)) < 1e-12
    tot = grm + 50000.0 ** 3 / 3 + 8 * 50000.0 ** 2 + 2 * 50000.0 * 600000
    assert abs(r["e2e_fp64_frac_of_peak"] - tot / 3.0 / (8 * 78.6e12)) < 1e-12
    assert bench.c3_split(600000, 8, 7) == (525000, 75000)
    assert bench.c3_split(10, 3, 2) == (8, 2)
