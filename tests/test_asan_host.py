"""AddressSanitizer + UndefinedBehaviorSanitizer over libgbm's host code (SURVEY.md §5 "Race
detection / sanitizers"): tools/asan_host.sh rebuilds the C-ABI shim and the kernels' host
launchers with host-only address + undefined-behaviour sanitizers (host only; GPU sanitizers are not available on this
pool) and runs tests/native/asan_driver.cpp — every binding entry point with bad arguments, the
no-device paths, and eight threads at once checking their thread-local error strings. CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not available")
def test_host_shim_clean_under_asan_ubsan(tmp_path):
    if shutil.which("nproc") is None:
        pytest.skip("no coreutils")
    env = dict(os.environ, ASAN_OUT=str(tmp_path))
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "asan_host.sh")], env=env, capture_output=True, text=True,
                       timeout=900)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "asan driver: 0 failures" in r.stdout, tail
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, tail
