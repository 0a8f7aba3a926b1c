"""Host C++ runtime under sanitizers. The TFRecord / Example / threaded
loader code (csrc/host) is compiled together with tests/native/host_selftest.cpp into a
standalone executable, once with AddressSanitizer + UndefinedBehaviorSanitizer and once with
ThreadSanitizer, and run on CPU: any sanitizer report or failed check fails the test.
(GPU-side sanitizers / XNACK are not available on the MI355X pool; kernels are covered by
bounds-checked host wrappers and the numerics tests instead.)"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "csrc", "host")
SRCS = [os.path.join(ROOT, "tests", "native", "host_selftest.cpp"), os.path.join(HOST, "tfrecord.cpp")]


def _build_and_run(tmp_path, flags, env_extra):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path / "host_selftest")
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-pthread", "-fno-omit-frame-pointer", "-I", HOST] + flags + SRCS + \
        ["-o", exe]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout
    env = dict(os.environ)
    env.update(env_extra)
    env.pop("LD_PRELOAD", None)  # the sanitizer runtime must come first
    r = subprocess.run([exe, str(tmp_path)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=300, env=env)
    out = r.stdout
    assert r.returncode == 0, out
    assert "all checks passed" in out, out
    for marker in ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer", "ERROR: LeakSanitizer"):
        assert marker not in out, out


def test_host_runtime_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
                   {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:verify_asan_link_order=0"})


def test_host_runtime_tsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"})
