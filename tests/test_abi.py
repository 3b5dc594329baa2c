"""CPU: the C-ABI library loads, exports every entry point that include/rtpt.h
declares, its struct layouts match rt_types.h, and argument errors come back
as status codes (no abort) — all without touching a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

import gpuraytracer_amd as g
from gpuraytracer_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "rtpt.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_\w+)\s*\(", text)))


def test_header_declares_expected_api():
    names = declared_symbols()
    for n in ["rt_create", "rt_set_seeds", "rt_fill_seeds", "rt_render", "rt_render_async",
              "rt_destroy", "rt_last_error", "rt_last_kernel_ms"]:
        assert n in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_native.library_path)
    missing = [n for n in declared_symbols() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(declared_symbols()) == set(_native.SIGNATURES), "binding table out of date"


def test_abi_version_and_status_strings():
    assert g.lib.rt_abi_version() == g.ABI_VERSION
    assert g.lib.rt_status_string(0) == b"RT_OK"
    assert g.lib.rt_status_string(5) == b"RT_ERR_STATE"


def test_struct_layout_matches_c_header():
    # sizes/offsets are asserted at import; spot-check a round trip through C
    s = g.Scene.cornell_box(40, 30)
    assert s.camera.resolution.x == 40 and s.camera.resolution.y == 30
    assert ctypes.sizeof(g.SphereGPU) == 80 and ctypes.sizeof(g.CameraGPU) == 64


def test_create_rejects_bad_descriptions_without_a_device():
    ctx = ctypes.c_void_p()
    assert g.lib.rt_create(None, ctypes.byref(ctx)) == 1
    assert b"null" in g.lib.rt_last_error(None)
    d = _native.SceneDesc()
    assert g.lib.rt_create(ctypes.byref(d), ctypes.byref(ctx)) == 1  # camera null
    assert not ctx.value


def test_null_context_calls_return_status():
    assert g.lib.rt_build_info(None, None) == 1
    assert g.lib.rt_render(None, None, None) == 1
    assert g.lib.rt_fill_seeds(None, 0) == 1
    assert g.lib.rt_destroy(None) == 0


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU node: covered by the gpu tests")
def test_no_device_is_reported_loudly():
    with pytest.raises(g.RtError) as e:
        g.Renderer(g.Scene.cornell_box(8, 8))
    assert e.value.status == 2  # RT_ERR_NO_DEVICE — no CPU fallback


def test_seed_helper_range():
    s = g.seed_splitmix(64, 32)
    assert s.shape == (32, 64) and s.dtype == np.uint32 and s.max() < 2**20


def test_scene_layout_uses_shared_edge_pairs():
    info = g.Scene.cornell_box(64, 48).describe()
    # four box clusters: the room (5 walls), the two rotated boxes, the light rectangle
    assert info == {"n_triangles": 36, "n_triangle_pairs": 18, "n_spheres": 0,
                    "lds_bytes": 18 * 112 + 4 * 112, "n_sphere_nodes": 0, "n_triangle_bvh_nodes": 0,
                    "n_box_clusters": 4, "pair_free_mask": 0, "sphere_kernel_lds_bytes": 0,
                    "kernel_layout": 6, "kernel_lds_bytes": 18 * 112 + 4 * 112 + 4 * 4679}
    boxes = g.Scene.random_boxes(16, 8, 4, seed=1).describe()
    assert boxes["n_box_clusters"] == 6 and boxes["pair_free_mask"] == 0  # room, 4 boxes, light
    soup = g.Scene.random_triangles(16, 8, 1000).describe()
    assert soup["n_triangle_bvh_nodes"] == 2 * 1036 - 1 and soup["lds_bytes"] == 0

    def bvh_nodes(n):  # median split, one sphere per leaf (rt_scene.cpp BvhBuild)
        return 1 if n <= 1 else 1 + bvh_nodes(n // 2) + bvh_nodes(n - n // 2)

    info = g.Scene.random_spheres(64, 48, 1000).describe()
    assert info["n_sphere_nodes"] == bvh_nodes(1000)
    assert info["n_triangle_pairs"] == 6
    # only the triangle pairs are staged (box clusters: triangle-only scenes);
    # the sphere BVH is read with scalar loads
    assert info["n_box_clusters"] == 2
    assert info["lds_bytes"] == 6 * 112
    # the compact sphere BVH (8 octant layouts x 1999 entries x 16 B, near/far
    # fp16 boxes) is read from global memory (L2): the compact-BVH kernel
    # stages only the pairs
    assert info["sphere_kernel_lds_bytes"] == 6 * 112
    big = g.Scene.random_spheres(16, 8, 5000).describe()
    assert big["lds_bytes"] == 6 * 112 and big["sphere_kernel_lds_bytes"] == 6 * 112
    assert big["n_sphere_nodes"] == bvh_nodes(5000)


# (scene, options) -> (kernel layout, dynamic LDS bytes the launcher requests):
# the bytes each layout's staging loops write, restated here from the kernels
# (rt_kernel.hip path_trace_kernel / path_trace_sorted_kernel, rt_free.hpp):
# pair records 112 B, single triangles 48 B, box clusters 112 B, Halton tables
# 4,679 floats, the sorted kernels' path buffers 1,097 float4 first.
PAIR, TRI, CLU, TAB, SORT = 112, 48, 112, 4 * 4679, 16 * 1097
LAYOUT_CASES = [
    ("cornell", {}, 6, 18 * PAIR + 4 * CLU + TAB),
    ("cornell", {"layout": "pairs"}, 1, 18 * PAIR),
    ("cornell", {"layout": "single"}, 0, 36 * TRI),
    ("cornell", {"layout": "global"}, 2, 0),
    ("cornell", {"layout": "pairsmem"}, 4, 0),
    ("cornell", {"layout": "sorted"}, 3, SORT + 18 * PAIR),
    ("cornell", {"layout": "bvh"}, 5, 0),
    ("spheres", {}, 7, 6 * PAIR),
    ("spheres", {"walk": "free"}, 8, 6 * PAIR),
    ("spheres", {"walk": "sorted"}, 10, SORT + 6 * PAIR),
    ("soup", {}, 5, 0),
    ("soup", {"walk": "free"}, 9, 0),
    ("soup", {"walk": "sorted"}, 11, SORT),
]


def layout_scene(name):
    return {"cornell": lambda: g.Scene.cornell_box(48, 32),
            "spheres": lambda: g.Scene.random_spheres(48, 32, 300, seed=3),
            "soup": lambda: g.Scene.random_triangles(48, 32, 1000)}[name]()


@pytest.mark.parametrize("name,opt,layout,lds", LAYOUT_CASES)
def test_kernel_layout_and_staged_lds_per_layout(name, opt, layout, lds):
    """rt_scene_describe_ex reports the launcher's own choice (rt::choose_kernel)
    and the dynamic LDS it requests, staged_lds_bytes: equal to what that
    layout's staging loops write (tests/test_gpu_parity.py checks
    rt_last_launch against it on the GPU)."""
    info = layout_scene(name).describe(g.Options(**opt))
    assert (info["kernel_layout"], info["kernel_lds_bytes"]) == (layout, lds), info


def test_create_options_are_validated_without_a_device():
    """rt_create_ex checks rt_create_options before it looks for a device:
    out-of-range values come back as RT_ERR_INVALID_ARG with a message."""
    ctx = ctypes.c_void_p()
    desc = g.Scene.cornell_box(8, 8).desc()
    o = _native.CreateOptions()
    g.lib.rt_create_options_default(ctypes.byref(o))
    assert bytes(o) == bytes(ctypes.sizeof(o))  # the defaults are all zero
    for field, bad in [("scene_layout", 7), ("lanes_per_pixel", 2), ("tri_bvh_build", 9),
                       ("tri_leaf_max", 129), ("sphere_leaf_max", 256), ("sphere_median", 2),
                       ("walk_scheduler", 4), ("walk_leaf_den", 65), ("tri_leaf_cost", -1.0)]:
        q = _native.CreateOptions()
        setattr(q, field, bad)
        assert g.lib.rt_create_ex(ctypes.byref(desc), ctypes.byref(q), ctypes.byref(ctx)) == 1, field
        assert field.encode() in g.lib.rt_last_error(None), field
        assert not ctx.value
    q = _native.CreateOptions()
    q.reserved[3] = 1
    assert g.lib.rt_create_ex(ctypes.byref(desc), ctypes.byref(q), ctypes.byref(ctx)) == 1
    assert b"reserved" in g.lib.rt_last_error(None)


def test_library_reads_no_environment():
    """Kernel-selecting knobs are rt_create_options fields: no object file of
    librtpt.so that is built from this repository's sources imports getenv.
    (rocPRIM's device sort in rt_lbvh.o reads ROCPRIM_USE_ATOMIC_BLOCK_ID, a
    switch of that third-party library's own block ordering.)"""
    import glob
    import subprocess
    objs = sorted(glob.glob(os.path.join(ROOT, "build", "*.o")))
    if not objs:
        pytest.skip("no build/ objects")
    users = []
    for o in objs:
        und = subprocess.run(["nm", "--undefined-only", o], capture_output=True, text=True).stdout
        if "getenv" in und:
            users.append(os.path.basename(o))
    assert users in ([], ["rt_lbvh.o"]), users
    src = "".join(open(f).read() for f in glob.glob(os.path.join(ROOT, "gpuraytracer_amd", "csrc", "*")))
    assert "getenv" not in src


def test_describe_follows_options_and_the_launcher():
    cornell = g.Scene.cornell_box(64, 48)
    forced = cornell.describe(g.Options(layout="bvh"))
    assert forced["n_triangle_bvh_nodes"] == 2 * 36 - 1 and forced["lds_bytes"] == 0
    # spheres with triangles that cannot be paired: the launcher takes the
    # single-record layout and the 32-B-node walks, not the one-wave sphere kernel
    sph = g.Scene.random_spheres(32, 16, 100)
    n = 11  # the 12 room/light triangles minus one: odd, no pair layout
    mats = (g.MaterialGPU * n)()
    verts = (g.float3 * (3 * n))()
    ctypes.memmove(ctypes.addressof(mats), ctypes.addressof(sph.materials), n * 48)
    ctypes.memmove(ctypes.addressof(verts), ctypes.addressof(sph.vertices), 3 * n * 16)
    odd = g.Scene(sph.camera, mats, verts, sph.light, sph.spheres)
    info = odd.describe()
    assert info["n_triangle_pairs"] == 0 and info["sphere_kernel_lds_bytes"] == 0
    assert sph.describe()["sphere_kernel_lds_bytes"] == 6 * 112
    # a forced layout also leaves the sphere kernel
    assert sph.describe(g.Options(layout="pairs"))["sphere_kernel_lds_bytes"] == 0


def test_options_from_env_is_explicit():
    """The RTPT_* variables reach a context only through Options.from_env()
    (bench.py and tools/); Renderer's default is the library's defaults."""
    env = {"RTPT_SCENE_MEM": "sorted", "RTPT_LANES": "16", "RTPT_TRI_BUILD": "lbvh",
           "RTPT_TRI_LEAF": "4", "RTPT_TRI_CT": "2.5", "RTPT_BVH_LEAF": "3", "RTPT_BVH_SAH": "0",
           "RTPT_WALK": "free"}
    o = g.Options.from_env(env)
    assert (o.layout, o.lanes, o.tri_build, o.tri_leaf_max, o.tri_leaf_cost, o.sphere_leaf_max,
            o.sphere_median, o.walk) == ("sorted", 16, "lbvh", 4, 2.5, 3, True, "free")
    c = o.c()
    assert (c.scene_layout, c.lanes_per_pixel, c.tri_bvh_build, c.walk_scheduler) == (5, 16, 2, 2)
    assert g.Options.from_env({}) == g.Options()


def _with_quads(base, n_quads, seed=3):
    """base's triangles + n_quads random planar quads (one shared-edge pair each)."""
    import ctypes
    rng = np.random.default_rng(seed)
    n0 = base.n_triangles
    n = n0 + 2 * n_quads
    mats = (g.MaterialGPU * n)()
    verts = (g.float3 * (3 * n))()
    ctypes.memmove(ctypes.addressof(mats), ctypes.addressof(base.materials), n0 * 48)
    ctypes.memmove(ctypes.addressof(verts), ctypes.addressof(base.vertices), 3 * n0 * 16)
    vv = np.frombuffer(verts, np.float32).reshape(-1, 4)
    mm = np.frombuffer(mats, np.float32).reshape(-1, 12)
    for q in range(n_quads):
        c = rng.uniform(-2.0, 2.0, 3)
        a, b = rng.normal(size=3) * 0.3, rng.normal(size=3) * 0.3
        P = [c, c + a, c + a + b, c + b]
        for t, tri in enumerate(((P[0], P[1], P[2]), (P[0], P[2], P[3]))):
            k = n0 + 2 * q + t
            vv[3 * k:3 * k + 3, :3] = np.array(tri, np.float32)
            mm[k, 0:3] = 0.5
            mm[k, 3] = 1.0
    return mats, verts


def test_sphere_kernel_pair_budget():
    """The one-wave sphere kernel stages the pair records in every workgroup, so
    it is taken only while they fit kSphPairLdsMaxBytes (6 KB, rt_kernel.hpp);
    above it the pair kernel (records shared by 256 threads) serves the scene."""
    base = g.Scene.cornell_box(64, 48)
    sph = g.Scene.random_spheres(64, 48, 200).spheres
    mixed = g.Scene(base.camera, base.materials, base.vertices, base.light, sph)
    info = mixed.describe()
    assert info["n_triangle_pairs"] == 18 and info["sphere_kernel_lds_bytes"] == 18 * 112
    mats, verts = _with_quads(base, 36)  # 54 pairs = 6048 B: still the sphere kernel
    at = g.Scene(base.camera, mats, verts, base.light, sph).describe()
    assert at["n_triangle_pairs"] == 54 and at["sphere_kernel_lds_bytes"] == 54 * 112
    mats, verts = _with_quads(base, 37)  # 55 pairs = 6160 B > 6 KB
    over = g.Scene(base.camera, mats, verts, base.light, sph).describe()
    assert over["n_triangle_pairs"] == 55 and over["sphere_kernel_lds_bytes"] == 0
    assert over["lds_bytes"] == 55 * 112


def test_portrait_resolution_is_rejected():
    """The reference computes aspect = float(res.x / res.y) in integers
    (sampling.metal:132): a portrait frame gives aspect 0 and halfHeight inf.
    The boundary refuses it with RT_ERR_INVALID_ARG instead (INTEGRATION.md
    §4, a documented deviation); square and landscape frames are accepted."""
    with pytest.raises(g.RtError) as e:
        g.Scene.cornell_box(30, 40).describe()
    assert e.value.status == 1 and "aspectRatio 0" in str(e.value)
    assert g.Scene.cornell_box(40, 40).describe()["n_triangles"] == 36
    assert g.Scene.cornell_box(41, 40).describe()["n_triangles"] == 36


def test_library_carries_the_tree_source_hash():
    """librtpt.so was built from exactly these sources (rt_build_sha, compiled
    in by the Makefile from gpuraytracer_amd/srchash.py); the loader refuses a
    mismatching binary."""
    from gpuraytracer_amd.srchash import kernel_source_sha
    assert g.lib.rt_build_sha().decode() == kernel_source_sha()


def test_last_launch_needs_a_render():
    info = _native.LaunchInfo()
    assert g.lib.rt_last_launch(None, ctypes.byref(info)) == 1


def _tonemap_inputs():
    rng = np.random.default_rng(3)
    v = np.concatenate([
        np.array([0.0, 1e-30, 6e-8, 1e-4, 0.05, 0.5, 1.0, 3.0, 65504.0, 65520.0, 1e6, np.inf],
                 np.float32),
        rng.exponential(0.3, 20000).astype(np.float32),
        rng.uniform(0, 50, 5000).astype(np.float32)])
    a = np.zeros((len(v), 4), np.float32)
    a[:, 0], a[:, 1], a[:, 2], a[:, 3] = v, v[::-1], np.roll(v, 7), 1.0
    return a


def test_host_tonemap_equals_oracle_tonemap():
    """rt_tonemap_rgba8 (host form of the kernel's RT_OUT_RGBA8 epilogue,
    rt::tonemap_channel) == the oracle's image.swift:35-65 restatement, incl.
    fp16 overflow (inf -> NaN after Reinhard -> 255, Swift min(1, NaN) = 1)."""
    import oracle_lib
    a = _tonemap_inputs()
    ours = g.tonemap_rgba8(a)
    assert np.array_equal(ours, oracle_lib.tonemap(a))
    assert ours[9, 0] == 255 and ours[11, 0] == 255  # 65520 and inf overflow fp16
    assert np.all(ours[:, 3] == 255)


def test_tonemap_contract_pow_vs_libm():
    """The contract's portable pow against float32 libm pow
    in a numpy restatement of image.swift:41-60: a byte can differ only where
    v*255 sits within the pow error of an integer."""
    a = _tonemap_inputs()[:, :3]
    v = a.astype(np.float16).astype(np.float32) * np.float32(2.0)
    with np.errstate(invalid="ignore"):
        v = v / (v + np.float32(1.0))
        p = np.power(v, np.float32(1.0) / np.float32(2.2))
    p = np.where(np.isnan(p), np.float32(1.0), np.clip(p, 0, 1))
    ref = (p * np.float32(255.0)).astype(np.uint8)
    ours = g.tonemap_rgba8(_tonemap_inputs())[:, :3]
    diff = ours.astype(int) - ref.astype(int)
    assert np.abs(diff).max() <= 1
    near = np.abs(p * 255.0 - np.round(p * 255.0)) < 1e-3
    assert np.all(near[diff != 0])


def test_comm_entry_points_reject_bad_arguments():
    """rt_comm_init / rt_render_gather / rt_comm_unique_id argument errors come
    back as status codes without a device (the RCCL calls are never reached)."""
    buf = (ctypes.c_uint8 * _native.RT_COMM_ID_BYTES)()
    assert g.lib.rt_comm_unique_id(None) == 1
    assert g.lib.rt_comm_init(None, 0, 1, buf) == 1
    assert g.lib.rt_render_gather(None, None, None, None) == 1
    assert b"null" in g.lib.rt_last_error(None)


def test_bench_multi_gpu_launcher_needs_the_gpus():
    """`bench.py --gpus N` outside torchrun spawns its own N ranks; with fewer
    visible GPUs it stops before spawning, with a clear message."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES=""))
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr


def test_c_program_links_the_abi(tmp_path):
    """A plain C99 program (what a Swift / cgo / JNI shim compiles against)
    includes rtpt.h, links librtpt.so and calls the host-only entry points:
    the tile layout of the multi-GPU gather and its host placement."""
    import shutil
    import subprocess
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    src = tmp_path / "abi.c"
    src.write_text(r'''
#include <stdio.h>
#include <string.h>
#include "rtpt.h"
int main(void) {
    rt_tile_layout_info a, b;
    if (rt_tile_layout(6, 5, 2, 0, 0, &a) || rt_tile_layout(6, 5, 2, 1, RT_OUT_RGBA8, &b)) return 1;
    if (a.rows != 3 || a.rows_max != 3 || a.row_bytes != 96 || a.tile_bytes != 288) return 2;
    if (b.rows != 2 || b.row_bytes != 24 || b.tile_bytes != 72) return 3;
    unsigned char g[2 * 72], f[5 * 24];
    for (int i = 0; i < (int)sizeof g; ++i) g[i] = (unsigned char)i;
    if (rt_place_tiles_host(g, 6, 5, 2, RT_OUT_RGBA8, f)) return 4;
    /* frame row 1 = rank 1's tile row 0, row 4 = rank 0's tile row 2 */
    if (memcmp(f + 24, g + 72, 24) || memcmp(f + 4 * 24, g + 48, 24)) return 5;
    if (rt_abi_version() != RTPT_ABI_VERSION) return 6;
    printf("ok\n");
    return 0;
}
''')
    exe = tmp_path / "abi"
    libdir = os.path.join(ROOT, "gpuraytracer_amd")
    subprocess.check_call([cc, "-std=c99", "-Wall", "-I", os.path.join(ROOT, "include"), str(src),
                           "-o", str(exe), "-L", libdir, "-lrtpt", "-Wl,-rpath," + libdir])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and out.stdout.strip() == "ok", (out.returncode, out.stderr[-500:])
