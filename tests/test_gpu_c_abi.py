"""GPU: a plain C99 program -- what a Swift, cgo or JNI shim compiles against --
renders through the C-ABI alone (no Python, no torch in the process):
rt_create_ex with options -> rt_fill_seeds -> rt_render -> rt_last_error on a
bad call -> rt_destroy.  Its fp32 frame is compared bit for bit with the
oracle.  The reference's only caller of this path is Renderer.draw()
(RTrace/renderer.swift:117-146), which a Swift host binds exactly like this
program."""
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle_lib
from gpuraytracer_amd import Scene, seed_splitmix
from test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

C_SRC = r'''
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "rtpt.h"

int main(int argc, char** argv) {
    const int W = atoi(argv[1]), H = atoi(argv[2]), spp = atoi(argv[3]);
    CameraGPU cam; MaterialGPU mats[RT_CORNELL_TRIANGLES]; rt_float3 verts[3 * RT_CORNELL_TRIANGLES];
    SquareLightGPU light; uint32_t nt = 0;
    if (rt_scene_cornell_box(W, H, &cam, mats, verts, &light, &nt) != RT_OK) return 10;
    rt_scene_desc d; memset(&d, 0, sizeof d);
    d.camera = &cam; d.materials = mats; d.square_lights = &light; d.n_square_lights = 1;
    d.vertices = verts; d.n_triangles = nt; d.device = 0;
    rt_create_options o; rt_create_options_default(&o);
    o.lanes_per_pixel = (uint32_t)atoi(argv[4]);
    rt_ctx* ctx = NULL;
    int st = rt_create_ex(&d, &o, &ctx);
    if (st != RT_OK) { fprintf(stderr, "create: %s\n", rt_last_error(NULL)); return 11; }
    if (rt_fill_seeds(ctx, 0x5EED00000000ull) != RT_OK) return 12;
    /* an invalid call: the status and the message, no abort */
    rt_render_params bad; memset(&bad, 0, sizeof bad);
    bad.spp = 1; bad.bounces = 9;
    if (rt_render(ctx, &bad, NULL) != RT_ERR_INVALID_ARG) return 13;
    if (strstr(rt_last_error(ctx), "bounces") == NULL) return 14;
    rt_render_params p; memset(&p, 0, sizeof p);
    p.spp = (uint32_t)spp; p.bounces = 3;
    float* img = (float*)malloc((size_t)W * H * 16);
    if ((st = rt_render(ctx, &p, img)) != RT_OK) { fprintf(stderr, "render: %s\n", rt_last_error(ctx)); return 15; }
    rt_launch_info li;
    if (rt_last_launch(ctx, &li) != RT_OK) return 16;
    FILE* f = fopen(argv[5], "wb");
    if (!f || fwrite(img, 16, (size_t)W * H, f) != (size_t)W * H) return 17;
    fclose(f);
    printf("%s\n", li.kernel);
    free(img);
    return rt_destroy(ctx);
}
'''


@pytest.fixture(scope="module")
def c_program(tmp_path_factory):
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    d = tmp_path_factory.mktemp("cabi")
    src = d / "render.c"
    src.write_text(C_SRC)
    exe = d / "render"
    libdir = os.path.join(ROOT, "gpuraytracer_amd")
    subprocess.check_call([cc, "-std=c99", "-Wall", "-I", os.path.join(ROOT, "include"), str(src),
                           "-o", str(exe), "-L", libdir, "-lrtpt", "-Wl,-rpath," + libdir])
    return str(exe), d


@pytest.mark.parametrize("lanes", [0, 4])
def test_c_program_renders_through_the_abi_bit_exact(c_program, lanes):
    exe, d = c_program
    W, H, spp = 48, 32, 12
    out = d / f"frame{lanes}.f32"
    r = subprocess.run([exe, str(W), str(H), str(spp), str(lanes), str(out)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stderr[-800:])
    assert r.stdout.startswith("rt::path_trace_kernel<3, 6,"), r.stdout  # the box-cluster kernel
    img = np.fromfile(out, np.float32).reshape(H, W, 4)
    s = Scene.cornell_box(W, H)
    ref = oracle_lib.render(s, seed_splitmix(W, H), spp, 3)
    assert_parity(img, ref, f"C program, lanes {lanes}")
