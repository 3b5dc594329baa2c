"""Diagnostic: which frame rows rt_place_tiles gets wrong (device frame)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch
from gpuraytracer_amd import RenderParams, Options, Renderer, Scene
from test_gpu_gather import _render_tiles
mode = sys.argv[1]
W, H = 1920, 1080
s = Scene.cornell_box(W, H)
with Renderer(s, options=Options.from_env()) as r:
    st = torch.cuda.current_stream()
    print("stream handle", st.cuda_stream)
    ref = r.render(RenderParams(spp=2))
    for world in (2, 3, 8):
        g = _render_tiles(r, s, world, 2, False, False, st)
        if mode == "sync":
            torch.cuda.synchronize()
        dev = torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0")
        r.place_tiles(g, world, out=dev, stream=st)
        if mode != "nohost":
            host = r.place_tiles(g, world)
        torch.cuda.synchronize()
        d = dev.cpu().numpy()
        bad = [y for y in range(H) if not np.array_equal(d[y].view(np.uint32), ref[y].view(np.uint32))]
        gh = g.cpu().numpy().view(np.float32).reshape(world, -1, W, 4)
        tb = [(k, j) for k in range(world) for j in range((H - 1 - k) // world + 1)
              if not np.array_equal(gh[k, j].view(np.uint32), ref[k + j * world].view(np.uint32))]
        print(mode, world, "dev bad rows", len(bad), bad[:12], "tile rows bad", len(tb), tb[:6])
        if bad:
            y = bad[0]
            cols = np.argwhere(np.any(d[y].view(np.uint32) != ref[y].view(np.uint32), axis=-1)).ravel()
            print("  row", y, "bad cols", len(cols), cols[:8], d[y, cols[0]], ref[y, cols[0]])
