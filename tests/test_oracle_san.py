"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer
(SURVEY.md §5 "Race detection / sanitizers"): `make -C oracle san` builds
oracle/cpu_ref.cpp with -fsanitize=address,undefined and
tests/cpp/oracle_san.cpp drives every entry point (kd-tree on ragged,
duplicate and lattice clouds, all five regularisations, LM and GN aligns,
linearize, compute_error, voxel grid, so3_exp, LDLT)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_clean_under_asan_ubsan():
    try:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "san"], check=True, capture_output=True,
                       timeout=300)
    except (subprocess.CalledProcessError, FileNotFoundError) as e:   # toolchain without the sanitizer runtimes
        pytest.skip(f"sanitizer build unavailable: {e}")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
               OMP_NUM_THREADS="2")
    r = subprocess.run([os.path.join(ROOT, "oracle", "_san", "oracle_san")], capture_output=True, text=True,
                       timeout=600, env=env)
    out = r.stdout + r.stderr
    assert "runtime error" not in out and "AddressSanitizer" not in out and "LeakSanitizer" not in out, out[-4000:]
    assert r.returncode == 0 and "oracle sanitizer run: ok" in out, out[-4000:]
