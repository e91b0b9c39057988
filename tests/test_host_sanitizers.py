"""Sanitizer builds of the native host runtime (SURVEY.md §5.2 race detection): the token loader's
producer/consumer ring under ThreadSanitizer, its mmap / copy loops under AddressSanitizer +
UBSan.  Host code only (GPU sanitizers are not available on the MI355X pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "pretraining_llm_amd", "csrc", "host")


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_token_loader_under_sanitizer(san, tmp_path):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = tmp_path / "loader_selftest"
    build = subprocess.run([cxx, "-O1", "-g", "-std=c++17", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-pthread",
                            os.path.join(HOST, "token_loader.cpp"), os.path.join(HOST, "selftest", "loader_selftest.cpp"),
                            "-o", str(exe)], capture_output=True, text=True, timeout=240)
    if build.returncode != 0 and "cannot find" in build.stderr and "san" in build.stderr:
        pytest.skip(f"sanitizer runtime for {san} not installed")
    assert build.returncode == 0, build.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="halt_on_error=1:detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(exe), str(tmp_path / "tokens.bin")], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0 and "loader_selftest ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-4000:]
