"""The library's host-only code (csrc/hybrd.cpp: fsolve's MINPACK hybrd as
scipy drives it; csrc/probes.cpp: the MT19937 binomial probe stream) under
AddressSanitizer + UndefinedBehaviorSanitizer: tools/asan_host.cpp drives
fsolve on converging, stalling, rootless and user-stopped systems and the
probe stream in split / whole draws at even and odd stream positions.  GPU
code cannot be sanitized on this pool; this covers the host code
the GPU path calls.  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_code_under_asan_ubsan(tmp_path):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "asan_host")
    csrc = os.path.join(ROOT, "sgvamp-py_amd", "csrc")
    cmd = [gxx, "-std=c++17", "-O1", "-g", "-Wno-psabi", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer",
           "-I" + os.path.join(ROOT, "include"), "-I" + csrc,
           os.path.join(ROOT, "tools", "asan_host.cpp"), os.path.join(csrc, "hybrd.cpp"),
           os.path.join(csrc, "probes.cpp"), "-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if b.returncode != 0 and "asan" in b.stderr.lower():
        pytest.skip("sanitizer runtime unavailable: " + b.stderr[-300:])
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert r.stdout.strip().endswith("ok"), r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
