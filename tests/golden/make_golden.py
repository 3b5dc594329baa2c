"""Generate the golden fixtures under tests/golden/ (committed with this script).

Each fixture holds the scene arrays (shaderTypes.h bytes), the seed texture,
the render parameters and the expected rgba32F image computed by the C oracle
(oracle/liboracle.so).  Before a fixture is written, the C oracle's image is
checked BIT-FOR-BIT against the independent numpy restatement
(oracle/pt_oracle_np.py); generation aborts on any difference.

The reference itself (Swift + Metal) cannot run here, so these
vectors pin the oracle's restatement, not a Metal run ("parity unpinned"
against Metal).  The only artefact the reference holds,
Sources/gpuRaytracer/example.png, is reduced to its light footprint
(footprint.json, by footprint_from_png()) and used as a geometry check.

Run:  python tests/golden/make_golden.py        (needs `make` first)
"""
import json
import os
import struct
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle_lib  # noqa: E402
import pt_oracle_mis_np  # noqa: E402
import pt_oracle_np  # noqa: E402
from gpuraytracer_amd import Scene  # noqa: E402


def scene_bytes(scene):
    d = dict(camera=np.frombuffer(bytes(scene.camera), np.uint8),
             materials=np.frombuffer(bytes(scene.materials), np.uint8),
             vertices=np.frombuffer(bytes(scene.vertices), np.uint8),
             light=np.frombuffer(bytes(scene.light), np.uint8))
    if scene.spheres is not None:
        d["spheres"] = np.frombuffer(bytes(scene.spheres), np.uint8)
    return d


def make(name, scene, seeds, spp, bounces, sample_base=0):
    out = oracle_lib.render(scene, seeds, spp, bounces, sample_base=sample_base)
    sc = pt_oracle_np.Scene(scene.camera, scene.materials, scene.light, scene.vertices,
                            scene.spheres)
    ref = pt_oracle_np.render(sc, seeds, spp, bounces, sample_base=sample_base)
    if not np.array_equal(out.view(np.uint32), ref.view(np.uint32)):
        bad = np.argwhere(out.view(np.uint32) != ref.view(np.uint32))
        raise SystemExit(f"{name}: C oracle != numpy restatement at {bad[:5].tolist()}")
    np.savez_compressed(os.path.join(HERE, name + ".npz"), seeds=seeds, out=out,
                        params=np.array([spp, bounces, sample_base], np.uint32),
                        **scene_bytes(scene))
    print(f"{name}: {out.shape} mean {out[..., :3].mean():.6f} (C == numpy, bit-exact)")


def make_mis(name, scene, camera_rays, mis_samples):
    """MIS integrator fixture: C oracle checked against pt_oracle_mis_np first."""
    out, out8 = oracle_lib.render_mis(scene, camera_rays, mis_samples)
    sc = pt_oracle_mis_np.Scene(scene.camera, scene.materials, scene.light, scene.vertices)
    ref, ref8 = pt_oracle_mis_np.render_mis(sc, camera_rays, mis_samples)
    if not (np.array_equal(out.view(np.uint32), ref.view(np.uint32)) and np.array_equal(out8, ref8)):
        raise SystemExit(f"{name}: C oracle != numpy MIS restatement")
    np.savez_compressed(os.path.join(HERE, name + ".npz"), out=out, out8=out8,
                        params=np.array([camera_rays, mis_samples], np.uint32),
                        **scene_bytes(scene))
    print(f"{name}: {out.shape} mean {out[..., :3].mean():.6f} (C == numpy, bit-exact)")


def read_png_rgba(path):
    """Tiny PNG decoder (8-bit RGB/RGBA, non-interlaced) for footprint extraction."""
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", None, None
    ctype = None
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        typ = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        if typ == b"IHDR":
            w, h, depth, ctype = struct.unpack(">IIBB", body[:10])
            assert depth == 8 and ctype in (2, 6)
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    bpp = 4 if ctype == 6 else 3
    raw = zlib.decompress(idat)
    stride = w * bpp
    img = np.zeros((h, stride), np.int32)
    prev = np.zeros(stride, np.int32)
    for y in range(h):
        f = raw[y * (stride + 1)]
        line = np.frombuffer(raw[y * (stride + 1) + 1:(y + 1) * (stride + 1)], np.uint8).astype(np.int32)
        cur = np.zeros(stride, np.int32)
        for x in range(stride):
            a = cur[x - bpp] if x >= bpp else 0
            b = prev[x]
            c = prev[x - bpp] if x >= bpp else 0
            if f == 0:
                v = line[x]
            elif f == 1:
                v = line[x] + a
            elif f == 2:
                v = line[x] + b
            elif f == 3:
                v = line[x] + (a + b) // 2
            else:
                p = a + b - c
                pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                v = line[x] + (a if pa <= pb and pa <= pc else (b if pb <= pc else c))
            cur[x] = v & 0xFF
        img[y] = cur
        prev = cur
    return img.reshape(h, w, bpp).astype(np.uint8)


def footprint_from_png():
    """Bounding box of the saturated light in the reference's example.png."""
    path = "/root/reference/Sources/gpuRaytracer/example.png"
    if not os.path.exists(path):
        print("reference PNG not present; footprint.json kept as is")
        return
    img = read_png_rgba(path)
    lum = img[..., :3].astype(np.int32).min(axis=-1)
    ys, xs = np.nonzero(lum >= 225)
    fp = dict(source="Sources/gpuRaytracer/example.png (reference, earlier revision)",
              width=int(img.shape[1]), height=int(img.shape[0]), threshold=225,
              rows=[int(ys.min()), int(ys.max())], cols=[int(xs.min()), int(xs.max())],
              corner_rgb=[int(v) for v in img[0, 0, :3]])
    with open(os.path.join(HERE, "footprint.json"), "w") as f:
        json.dump(fp, f, indent=1)
    print("footprint:", fp)


def main():
    key = 0x5EED00000000
    s = Scene.cornell_box(16, 16)
    make("cornell_16x16_s4_b3", s, oracle_lib.seeds(16, 16, key), 4, 3)
    s = Scene.cornell_box(128, 128)
    make("cornell_128x128_s1_b3", s, oracle_lib.seeds(128, 128, key), 1, 3)
    # full-range u32 seeds (wrap-around of seed + n) and 4 bounces, odd size
    rng = np.random.default_rng(7)
    s = Scene.cornell_box(24, 13)
    sd = rng.integers(0, 2**32, size=(13, 24), dtype=np.uint64).astype(np.uint32)
    sd[0, :4] = [0, 0xFFFFFFFF, 0xFFFFFFFE, 2**20 - 1]
    make("cornell_24x13_s3_b4_u32seeds", s, sd, 3, 4, sample_base=5)
    s = Scene.random_spheres(16, 16, 60, seed=42)
    make("spheres60_16x16_s2_b3", s, oracle_lib.seeds(16, 16, key), 2, 3)
    make_mis("mis_16x12_c2_m12", Scene.cornell_box_mis(16, 12), 2, 12)
    footprint_from_png()


if __name__ == "__main__":
    main()
