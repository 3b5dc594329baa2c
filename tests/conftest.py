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


def _ensure_built():
    need = [os.path.join(ROOT, "gpuraytracer_amd", "librtpt.so"),
            os.path.join(ROOT, "oracle", "liboracle.so")]
    if not all(os.path.exists(p) for p in need):
        subprocess.check_call(["make", "-C", ROOT, "-j8"], stdout=subprocess.DEVNULL)


_ensure_built()
