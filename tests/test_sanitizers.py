"""CPU: the host build of the bitboard core + the C oracle under ASan / UBSan (SURVEY.md §5
"Race detection/sanitizers").  GPU sanitizers are not available on this pool, so the device
logic (gc_core.h / gc_env.h / gc_fide.h) is sanitized in its host form, on a seeded
differential run against the oracle (tests/core_host/sanitize_main.cpp)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="needs gcc / g++")
def test_core_and_oracle_under_asan_ubsan(tmp_path):
    obj = tmp_path / "oracle.o"
    exe = tmp_path / "sanitize"
    subprocess.run(["gcc", "-std=c11", "-c", *SAN, "-o", str(obj), os.path.join(ROOT, "oracle", "gc_oracle.c")],
                   check=True)
    subprocess.run(["g++", "-std=c++17", "-Wno-unknown-pragmas", *SAN, "-o", str(exe),
                    os.path.join(ROOT, "tests", "core_host", "sanitize_main.cpp"), str(obj), "-lpthread"], check=True)
    # verify_asan_link_order=0: the runtime need not come first in the library list (the
    # environment may preload its own libraries)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), "300"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "fails 0" in r.stdout
