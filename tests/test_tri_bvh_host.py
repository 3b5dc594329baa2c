"""CPU: the host binned-SAH triangle BVH (rt_scene.cpp build_tri_sah, exported
by librtpt.so) checked by a small C++ program linked against the library:
perm / leaf-order records, every triangle in exactly one leaf per octant
layout, escapes inside the layout, every box a superset of its subtree and of
its triangles padded by the margin, and the stackless closest-hit walk of each
octant layout equal to brute force on 4000 random rays (exact duplicates
included: ties to the lower id).  The GPU walks over the same layout are the
parity tests (tests/test_gpu_parity.py::test_triangle_bvh_gpu_build_bit_exact)."""
import os
import shutil
import subprocess

import pytest

from conftest import native_toolchain

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        pytest.skip("no C++ compiler")
    out = tmp_path_factory.mktemp("bvh") / "tri_bvh_check"
    cxx, san, lib = native_toolchain(cxx)
    subprocess.check_call([cxx, "-std=c++17", "-O2", *san, "-I", os.path.join(ROOT, "include"),
                           "-I", os.path.join(ROOT, "gpuraytracer_amd", "csrc"),
                           os.path.join(ROOT, "tests", "native", "tri_bvh_check.cpp"),
                           "-L", lib, "-lrtpt", f"-Wl,-rpath,{lib}", "-o", str(out)])
    return str(out)


@pytest.mark.parametrize("n,seed,dup,leaf", [(3000, 1, 0, None), (2500, 2, 1, None), (3000, 3, 0, "4")])
def test_host_sah_triangle_bvh_layout_and_walks(checker, n, seed, dup, leaf):
    args = [checker, str(n), str(seed), str(dup)] + ([leaf, "2"] if leaf else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
