"""gpuraytracer_amd — MI355X-native drop-in for the ``pathTrace`` hot path of
Nishad-Sharma/gpuRaytracer.

The product is ``librtpt.so`` (HIP kernel for gfx950 + the C-ABI of
``include/rtpt.h``).  This package is the Python host mirror of the
reference's Swift host API, used by the tests and ``bench.py``:

* :class:`Scene` — ``RTrace/scene.swift`` (``initCornellBox`` and the
  config-4 sphere field), holding the ``shaderTypes.h`` arrays.
* :class:`Renderer` — ``RTrace/renderer.swift`` (``init`` uploads the scene and
  the seed texture, ``draw`` dispatches and waits).

There is no CPU fallback: importing fails loudly when ``librtpt.so`` has not
been built (``make`` or ``__graft_entry__.build()``), and rendering fails
loudly without a HIP device.
"""
from __future__ import annotations

from ._native import (ABI_VERSION, CameraGPU, MaterialGPU, RtError, SphereGPU,
                      SquareLightGPU, float3, lib, library_path)
from .host import (DEFAULT_SEED_KEY, MisParams, Options, RenderParams, Renderer, Scene, comm_unique_id,
                   place_tiles_host, seed_splitmix, tile_layout, tonemap_rgba8)

__all__ = [
    "ABI_VERSION", "CameraGPU", "MaterialGPU", "SphereGPU", "SquareLightGPU", "float3",
    "RtError", "lib", "library_path", "Scene", "Renderer", "RenderParams", "MisParams",
    "DEFAULT_SEED_KEY", "seed_splitmix", "tonemap_rgba8", "comm_unique_id", "tile_layout",
    "place_tiles_host",
]
