"""GPU: the C++ host of record (gpuraytracer_amd/rtrace, the mirror of
RTrace/main.swift + Renderer) run as a child process, its files checked
against the oracle.

* PNG: the kernel's fused RGBA8 store (RT_OUT_RGBA8) = the oracle render
  tonemapped by the oracle (image.swift:35-65), byte for byte.
* PFM (--pfm): the fp32 frame, bit-exact against the oracle.
* --mis: the SwiftPM drawTriangle integrator; PNG = the kernel's own RGBA8,
  PFM = its radiance sums, both against the oracle.
"""
import os
import struct
import subprocess
import zlib

import numpy as np
import pytest

import oracle_lib
from gpuraytracer_amd import Scene, seed_splitmix
from test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RTRACE = os.path.join(ROOT, "gpuraytracer_amd", "rtrace")


def read_png_rgba8(path):
    """Decoder for 8-bit RGBA PNGs with filter type 0 rows (what rtrace writes)."""
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat = 8, b""
    w = h = None
    while pos < len(data):
        n, kind = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        if kind == b"IHDR":
            w, h, depth, ctype = struct.unpack(">IIBB", body[:10])
            assert (depth, ctype) == (8, 6)
        elif kind == b"IDAT":
            idat += body
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + 4 * w)
    assert np.all(raw[:, 0] == 0)
    return raw[:, 1:].reshape(h, w, 4)


def read_pfm(path):
    with open(path, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = (int(v) for v in f.readline().split())
        assert float(f.readline()) < 0  # little endian
        a = np.frombuffer(f.read(), "<f4").reshape(h, w, 3)
    return a[::-1]  # PFM stores the bottom row first


def run(*args):
    r = subprocess.run([RTRACE, *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return r.stdout


@pytest.mark.parametrize("batch", [None, "3"])
def test_rtrace_png_and_pfm_vs_oracle(tmp_path, batch):
    W, H, spp = 64, 48, 8
    extra = ["--batch", batch] if batch else []
    png, pfm = str(tmp_path / "out.png"), str(tmp_path / "out.pfm")
    png2 = str(tmp_path / "fused.png")
    run(png, "--res", f"{W}x{H}", "--spp", str(spp), "--pfm", pfm, *extra)
    run(png2, "--res", f"{W}x{H}", "--spp", str(spp), *extra)  # no --pfm: fused RGBA8
    s = Scene.cornell_box(W, H)
    ref = oracle_lib.render(s, seed_splitmix(W, H), spp, 3)
    assert_parity(read_pfm(pfm), ref[..., :3], "rtrace --pfm")
    ref8 = oracle_lib.tonemap(ref)
    assert np.array_equal(read_png_rgba8(png), ref8)
    assert np.array_equal(read_png_rgba8(png2), ref8)


def test_rtrace_mis_vs_oracle(tmp_path):
    W, H = 48, 32
    png, pfm = str(tmp_path / "mis.png"), str(tmp_path / "mis.pfm")
    run("--mis", png, "--res", f"{W}x{H}", "--camera-rays", "2", "--mis-samples", "12",
        "--pfm", pfm)
    s = Scene.cornell_box_mis(W, H)
    out, out8 = oracle_lib.render_mis(s, camera_rays=2, mis_samples=12)
    assert_parity(read_pfm(pfm), out[..., :3], "rtrace --mis sums")
    assert np.array_equal(read_png_rgba8(png), out8)


def test_rtrace_rejects_bad_arguments():
    r = subprocess.run([RTRACE, "--res", "bogus"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2
    r = subprocess.run([RTRACE, "--mis", "--scene", "spheres:10"], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 2
