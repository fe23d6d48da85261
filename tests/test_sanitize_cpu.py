"""AddressSanitizer + UBSan run of the host-side C++ of the C ABI
(csrc/ace_host.cpp) and of the oracle's C restatement (oracle/ace_ref.c)
through tests/sanitize_host.cpp (sanitizers on host code; GPU
sanitizers are not available on this pool).  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def test_host_code_is_sanitizer_clean(tmp_path):
    gxx = shutil.which("g++")
    gcc = shutil.which("gcc")
    if not gxx or not gcc:
        pytest.skip("no host compiler")
    flags = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
             "-fno-sanitize-recover=all"]
    ref_o = str(tmp_path / "ace_ref.o")
    subprocess.run([gcc, *flags, "-std=c11", "-D_GNU_SOURCE", "-ffp-contract=off", "-c",
                    os.path.join(ROOT, "oracle", "ace_ref.c"), "-o", ref_o], check=True)
    exe = str(tmp_path / "sanitize_host")
    subprocess.run([gxx, *flags, "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "sanitize_host.cpp"),
                    os.path.join(ROOT, "additivecausalexpansion_amd", "csrc", "ace_host.cpp"),
                    ref_o, "-o", exe, "-lm"], check=True)
    # verify_asan_link_order=0: the process environment may preload other
    # libraries ahead of the ASan runtime; that is not a finding
    env = dict(os.environ,
               ASAN_OPTIONS="halt_on_error=1:detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    out = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "sanitize_host: OK" in out.stdout
