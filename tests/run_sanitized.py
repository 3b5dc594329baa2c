#!/usr/bin/env python3
"""Run the CPU tests of the library's host C++ and of the oracle under
AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5 "Race detection /
sanitizers"): `make asan-test`, or tests/test_sanitizers.py in the CPU suite.

The sanitized libraries come from `make asan` (build_asan/): the scene
compile and the host BVH builds (rt_scene.cpp, several host threads), the
C-ABI host paths and the tile layout / host placement (rt_api.cpp), the image
epilogue (rt_image.cpp) and the oracle (pt_oracle.c).  The test processes
preload clang's ASan runtime (python itself is not instrumented); the C++
checkers of tests/native/ are compiled with the same flags.  Any ASan report
or UBSan finding aborts the process, which fails the run.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = ["tests/test_tri_bvh_host.py", "tests/test_cluster_host.py", "tests/test_multirank.py",
         "tests/test_oracle.py", "tests/test_abi.py"]


def main(extra):
    san_dir = os.environ.get("RTPT_SAN_DIR") or os.path.join(ROOT, "build_asan")
    rt = os.environ.get("RTPT_SAN_RT") or subprocess.check_output(
        ["/opt/rocm/llvm/bin/clang++", "-print-file-name=libclang_rt.asan-x86_64.so"], text=True).strip()
    env = dict(os.environ)
    env.update({
        "LD_PRELOAD": rt,
        "ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1:abort_on_error=1:detect_odr_violation=0",
        "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1",
        "RTPT_SAN_DIR": san_dir,
        "RTPT_LIB": os.path.join(san_dir, "librtpt.so"),
        "RTPT_ORACLE_LIB": os.path.join(san_dir, "liboracle.so"),
    })
    cmd = [sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu", "-p", "no:cacheprovider",
           *TESTS, *extra]
    return subprocess.call(cmd, cwd=ROOT, env=env)


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
