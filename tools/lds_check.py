#!/usr/bin/env python3
"""Run every kernel layout of tests/test_abi.py LAYOUT_CASES through an
-DRT_LDS_CHECK build (RTPT_LIB=abvar/librtpt_ldschk.so): each kernel compares
the end of its staging loops with its dispatch's dynamic LDS, and rt_render
fails with RT_ERR_LAUNCH "LDS overflow" when it does not fit.  With
--expect-overflow (the RT_LDS_UNDERSIZE negative control, which requests one
float4 less) every layout that stages anything must fail that way instead.

    tools/lds_check.py [--expect-overflow] [out.json]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: F401,E402  (one HIP runtime)
from gpuraytracer_amd import Options, RenderParams, Renderer, RtError, seed_splitmix  # noqa: E402
from test_abi import LAYOUT_CASES, layout_scene  # noqa: E402

expect = "--expect-overflow" in sys.argv
args = [a for a in sys.argv[1:] if not a.startswith("--")]
rows, ok = [], True
for name, opt, layout, lds in LAYOUT_CASES:
    s = layout_scene(name)
    row = {"scene": name, "options": opt, "layout": layout, "lds": lds}
    try:
        with Renderer(s, seeds=seed_splitmix(48, 32), options=Options(**opt)) as r:
            r.render(RenderParams(spp=2, bounces=3))
            row["launch_lds"] = r.last_launch()["lds_bytes"]
        row["result"] = "ok"
    except RtError as e:
        row["result"] = str(e)
    overflow = "LDS overflow" in row["result"]
    good = (overflow == (lds > 0)) if expect else row["result"] == "ok"
    row["as_expected"] = good
    ok = ok and good
    rows.append(row)
    print(json.dumps(row))
out = {"expect_overflow": expect, "all_as_expected": ok, "cases": rows}
if args:
    open(args[0], "w").write(json.dumps(out, indent=1))
sys.exit(0 if ok else 1)
