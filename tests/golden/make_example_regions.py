#!/usr/bin/env python3
"""Radiance fixture from the reference's only rendered artefact.

    python tests/golden/make_example_regions.py [/root/reference]

Writes ``tests/golden/example_png_regions.json``: the mean 8-bit RGB of
``Sources/gpuRaytracer/example.png`` (800x600, the README's image, README.md:1)
over each surface of the live Cornell scene, the surfaces being the oracle's
primary-hit ids through the pixel centres (``region_masks`` below, shared with
tests/test_oracle.py), each eroded by 4 px so that the PNG's silhouettes (the
image is an earlier revision, a pixel or two off in places) do not mix
neighbouring surfaces.  Data measured from the image; no reference source.

tests/test_oracle.py::test_radiance_vs_reference_example_png compares the
oracle's render of the same frame against these means: it pins the NEE
radiance scale (white/grey surfaces) and records why radiance parity cannot
be pinned further (the coloured walls).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))

# primary ids of RTrace/scene.swift's triangles (Appendix B of SURVEY.md)
REGIONS = {
    "back_wall": (0, 1),       # scene.swift:81-90
    "red_wall": (2, 3),        # :93-102
    "green_wall": (4, 5),      # :105-114
    "floor": (6, 7),           # :117-126
    "ceiling": (8, 9),         # :129-138
    "tall_box": tuple(range(10, 22)),
    "short_box": tuple(range(22, 34)),
    "light": (34, 35),         # :58-59
}
ERODE = 4


def region_masks(ids):
    """{name: bool (600, 800)} -- pixels whose primary hit is the region, at
    least ERODE px (Chebyshev) away from any pixel of another region."""
    from scipy.ndimage import binary_erosion
    out = {}
    for name, group in REGIONS.items():
        m = np.isin(ids, group)
        out[name] = binary_erosion(m, structure=np.ones((2 * ERODE + 1, 2 * ERODE + 1), bool))
    return out


def main(ref_root):
    from PIL import Image
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    from gpuraytracer_amd import Scene
    png = os.path.join(ref_root, "Sources", "gpuRaytracer", "example.png")
    im = np.array(Image.open(png))[..., :3].astype(np.float64)
    assert im.shape == (600, 800, 3)
    ids = oracle_lib.primary_ids(Scene.cornell_box(800, 600))
    res = {}
    for name, m in region_masks(ids).items():
        res[name] = {"pixels": int(m.sum()), "mean_rgb": [round(float(v), 3) for v in im[m].mean(axis=0)]}
    out = os.path.join(HERE, "example_png_regions.json")
    json.dump({"source": "Sources/gpuRaytracer/example.png (800x600 RGBA8)", "erode_px": ERODE,
               "regions": res}, open(out, "w"), indent=1)
    print(out, json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
