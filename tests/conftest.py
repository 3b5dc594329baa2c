"""Shared test setup.

``gpu``-marked tests need a real MI355X and call the HIP path through the
C-ABI (librtpt.so); everything else runs on the CPU: the oracle against the
golden fixtures and known answers, the host logic, the ABI surface, and the
multi-rank tiling with gloo.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) — run with -m gpu")


def native_toolchain(cxx):
    """(compiler, extra flags, librtpt directory) for the tests' small C++
    checkers: the plain build, or under tests/run_sanitized.py (RTPT_SAN_DIR)
    clang++ with ASan/UBSan linked against the sanitizer build (make asan)."""
    san_dir = os.environ.get("RTPT_SAN_DIR")
    if not san_dir:
        return cxx, [], os.path.join(ROOT, "gpuraytracer_amd")
    flags = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
             "-g", "-shared-libasan"]
    return "/opt/rocm/llvm/bin/clang++", flags, san_dir


def _lib_is_fresh(path):
    """Whether the built librtpt.so carries this tree's source hash (its
    rt_build_sha() string), read from the file's bytes: loading it here would
    map a HIP runtime before the tests choose one."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "_rt_srchash", os.path.join(ROOT, "gpuraytracer_amd", "srchash.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)  # not via the package: that would load the library
    kernel_source_sha = mod.kernel_source_sha
    with open(path, "rb") as f:
        return b"\0" + kernel_source_sha().encode() + b"\0" in f.read()


def _ensure_built():
    lib = os.path.join(ROOT, "gpuraytracer_amd", "librtpt.so")
    need = [lib, os.path.join(ROOT, "oracle", "liboracle.so")]
    fresh = all(os.path.exists(p) for p in need) and _lib_is_fresh(lib)
    if not fresh:  # missing, or built from other sources than this tree
        subprocess.check_call(["make", "-C", ROOT, "-j8"], stdout=subprocess.DEVNULL)
    orc = os.path.join(ROOT, "oracle")
    if os.path.getmtime(os.path.join(orc, "pt_oracle.c")) > os.path.getmtime(need[1]):
        subprocess.check_call(["make", "-C", orc], stdout=subprocess.DEVNULL)


_ensure_built()
