"""CPU: the container shrink of the box clusters (rt_scene.cpp build_clusters,
DESIGN.md §3.12) checked by a small C++ program linked against librtpt.so and
the oracle: random shadow / light-sample segments that pass the kernel's
container test (both ends strictly inside the stored shrunk room, e = o + d*tmax
in the kernel's float order; half of them with an end within a few ulps of a
shrunk plane) have no accepted hit on any room triangle under the reference's
triangle test -- so skipping the room for them cannot change a result.  A
negative control grows the box by 2e-4 and must find such a hit.  The GPU side
is covered by the parity tests (tests/test_gpu_parity.py, tests/test_gpu_mis.py)."""
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
    cxx, san, lib = native_toolchain(cxx)
    orc = os.environ.get("RTPT_SAN_DIR") or os.path.join(ROOT, "oracle")
    if not os.path.exists(os.path.join(orc, "liboracle.so")):
        pytest.skip("oracle/liboracle.so not built")
    out = tmp_path_factory.mktemp("clu") / "cluster_check"
    subprocess.check_call([cxx, "-std=c++17", "-O2", "-ffp-contract=off", *san, "-I", os.path.join(ROOT, "include"),
                           "-I", os.path.join(ROOT, "gpuraytracer_amd", "csrc"),
                           os.path.join(ROOT, "tests", "native", "cluster_check.cpp"),
                           "-L", lib, "-lrtpt", f"-Wl,-rpath,{lib}",
                           "-L", orc, "-loracle", f"-Wl,-rpath,{orc}", "-o", str(out)])
    return str(out)


@pytest.mark.parametrize("mis,seed", [(0, 1), (0, 2), (1, 3)])
def test_container_shrink_is_conservative(checker, mis, seed):
    r = subprocess.run([checker, str(mis), str(seed)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr


def test_container_check_catches_a_wider_box(checker):
    r = subprocess.run([checker, "1", "1", "0.0002"], capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "hits triangle" in r.stdout, r.stdout + r.stderr
