"""CPU: the host C++ of librtpt.so and the oracle under ASan + UBSan (SURVEY
§5).  `make asan` builds the sanitized libraries; tests/run_sanitized.py runs
the CPU tests of that code with them (host BVH builds on host threads, box
clusters, tile layout and placement, the oracle, the C-ABI argument paths).
A negative control proves the instrumentation is live: a placement into a
frame one row too small must stop with ASan's heap-buffer-overflow report."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/llvm/bin/clang++"

pytestmark = pytest.mark.skipif(not os.path.exists(CLANG) or shutil.which("make") is None,
                                reason="needs ROCm's clang and make")


@pytest.fixture(scope="module")
def san_env():
    subprocess.check_call(["make", "-C", ROOT, "-j8", "asan"], stdout=subprocess.DEVNULL)
    rt = subprocess.check_output([CLANG, "-print-file-name=libclang_rt.asan-x86_64.so"], text=True).strip()
    d = os.path.join(ROOT, "build_asan")
    return dict(os.environ, RTPT_SAN_DIR=d, RTPT_SAN_RT=rt)


def test_cpu_suite_clean_under_asan_ubsan(san_env):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "run_sanitized.py")], env=san_env,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert " passed" in r.stdout and "failed" not in r.stdout


def test_asan_catches_an_overflow_in_the_library(san_env):
    code = r'''
import ctypes, numpy as np
lib = ctypes.CDLL("%s")
W, H, N = 16, 9, 2
g = np.zeros(N * 5 * W * 4, np.float32)      # 2 tiles of 5 rows (rows_max = 5)
frame = np.zeros((H - 1) * W * 4, np.float32)  # one row short
lib.rt_place_tiles_host(g.ctypes.data_as(ctypes.c_void_p), W, H, N, 0, frame.ctypes.data_as(ctypes.c_void_p))
print("no report")
''' % os.path.join(san_env["RTPT_SAN_DIR"], "librtpt.so")
    env = dict(san_env, LD_PRELOAD=san_env["RTPT_SAN_RT"],
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:detect_odr_violation=0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "heap-buffer-overflow" in r.stderr, (r.returncode, r.stderr[-2000:])
    assert "rt_place_tiles_host" in r.stderr
