"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer
(SURVEY.md §5).  The reference has undefined behaviour on the hot path --
SetPixel's index+3 store on RGB contexts runs one double past the buffer at
the last pixel (cpp:510, Appendix A.6), RGB textures leave the sampled alpha
uninitialised (cpp:571-573, used at cpp:746,773, A.2) -- which the oracle
restates as defined behaviour.  This runs the oracle's own CPU tests (the
Appendix-A known answers, the golden fixtures, the reference-binding
fixtures, the triangle rules, the audio DSP and the command-list scenes)
against `oracle/build/liboracle_san.so` (make -C oracle san) in a child
Python with the ASan runtime preloaded, and checks first that the sanitizer
is live (a deliberate overflow through the same library must abort)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime():
    if shutil.which("gcc") is None:
        return None
    out = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    return out if os.path.isabs(out) and os.path.exists(out) else None


@pytest.fixture(scope="module")
def san_env():
    rt = _runtime()
    if rt is None:
        pytest.skip("gcc's ASan runtime is not installed")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "san"], check=True)
    env = dict(os.environ)
    env.update(LD_PRELOAD=rt, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               NR_ORACLE_SO=os.path.join(ROOT, "oracle", "build", "liboracle_san.so"))
    return env


CANARY = r"""
import sys
sys.path.insert(0, %r); sys.path.insert(0, %r)
import numpy as np, ctypes, scenes
ctx = scenes.OracleFactory().context(16, 16, False)
ctx.set_color(0.5, 0.5, 0.5, 0.5)
small = np.zeros(8, dtype=np.float64)            # the frame needs 16*16*3 doubles
ctx.lib.GetBuffer(ctx._ptr, small.ctypes.data_as(ctypes.c_void_p))
print("NOT CAUGHT")
""" % (ROOT, os.path.join(ROOT, "tests"))


def test_sanitizer_is_live(san_env):
    r = subprocess.run([sys.executable, "-c", CANARY], env=san_env, capture_output=True, text=True, timeout=300)
    assert "NOT CAUGHT" not in r.stdout
    assert "AddressSanitizer" in r.stderr and "heap-buffer-overflow" in r.stderr, r.stderr[-2000:]


def test_oracle_cpu_suite_is_clean_under_asan_ubsan(san_env):
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "not gpu", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_oracle.py"), os.path.join(ROOT, "tests", "test_audio.py"),
                        os.path.join(ROOT, "tests", "test_command_list.py")],
                       env=san_env, capture_output=True, text=True, timeout=900, cwd=ROOT)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, tail
    assert " passed" in r.stdout, tail
