#!/usr/bin/env python3
"""Geometry fixture from the reference's only rendered artefact.

    python tests/golden/make_example_masks.py [/root/reference]

Reads ``Sources/gpuRaytracer/example.png`` (the README's image, README.md:1:
an 800x600 tonemapped render of an earlier revision of the same Cornell
scene) and writes ``tests/golden/example_png_geometry.npz`` -- data measured
from the image, no reference source:

* ``cls``: per-pixel class by colour, 0 = black (the camera sees past the open
  front, no hit), 1 = red wall, 2 = green wall, 3 = the light (emissive
  overwrite, saturated white), 4 = anything else (grey surfaces).  Thresholds
  are strict (a wall's other channels are exactly 0 in the image) so that the
  red/green colour bleeding onto the boxes stays grey.
* ``row_edges`` / ``col_edges``: (line, position) of every luminance step of at
  least EDGE_THRESHOLD along rows 40, 50, ..., 570 (columns 40, ..., 770), after
  a 5x5 median (the image is noisy) and a 9-pixel box filter along the line's
  normal; local maxima within +-3 px.  These are the silhouettes and creases
  the image shows: walls, floor and ceiling lines, both boxes, the light --
  plus the floor's shadow boundaries, which no geometry produces.

The radiance of this earlier revision is NOT a fixture; only
where things are.  tests/test_oracle.py checks the oracle's primary-hit ids of
the live scene against it.
"""
import os
import sys

import numpy as np

EDGE_THRESHOLD = 6.0
HERE = os.path.dirname(os.path.abspath(__file__))


def step_peaks(profile, thr):
    g = np.abs(np.diff(profile))
    out = []
    for x in range(3, len(g) - 3):
        if g[x] >= thr and g[x] == g[x - 3:x + 4].max():
            out.append(x + 1)  # first pixel past the step
    return out


def main(ref_root):
    from PIL import Image
    from scipy.ndimage import median_filter, uniform_filter
    png = os.path.join(ref_root, "Sources", "gpuRaytracer", "example.png")
    im = np.array(Image.open(png))[..., :3].astype(np.int32)
    assert im.shape == (600, 800, 3)
    R, G, B = im[..., 0], im[..., 1], im[..., 2]
    cls = np.full((600, 800), 4, np.uint8)
    cls[(R < 8) & (G < 8) & (B < 8)] = 0
    cls[(G < 8) & (B < 8) & (R > 30)] = 1
    cls[(R < 8) & (B < 8) & (G > 30)] = 2
    cls[(R >= 225) & (G >= 225) & (B >= 225)] = 3
    base = median_filter(im.mean(axis=2), size=5)
    smh = uniform_filter(base, size=(9, 3))
    smv = uniform_filter(base, size=(3, 9))
    row_edges = [(y, x) for y in range(40, 580, 10) for x in step_peaks(smh[y], EDGE_THRESHOLD)]
    col_edges = [(x, y) for x in range(40, 780, 10) for y in step_peaks(smv[:, x], EDGE_THRESHOLD)]
    out = os.path.join(HERE, "example_png_geometry.npz")
    np.savez_compressed(out, cls=cls, row_edges=np.array(row_edges, np.int16),
                        col_edges=np.array(col_edges, np.int16),
                        edge_threshold=np.float32(EDGE_THRESHOLD))
    print(f"{out}: {len(row_edges)} row edges, {len(col_edges)} column edges, "
          f"class counts {np.bincount(cls.ravel(), minlength=5).tolist()}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
