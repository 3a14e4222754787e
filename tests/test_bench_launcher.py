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
