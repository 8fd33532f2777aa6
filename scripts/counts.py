#!/usr/bin/env python3
"""Per-launch event counts of the counting kernel variant (dev tool).

usage: counts.py [scene W H SPP] ...   (defaults: the three A/B scenes)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd")]
import torch  # noqa: E402

import rtgo  # noqa: E402

sc = os.path.join(ROOT, "scenes")
cases = [("facing", os.path.join(sc, "sphere_reflections_light_facing.json"), 800, 600, 100),
         ("silver", os.path.join(sc, "final_silver_prism_purple_cube_facing.json"), 1200, 900, 100)]
if len(sys.argv) > 4:
    cases = [(sys.argv[1], sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))]


def load(path):
    if path == "spheres10k":  # config C4/C5 scene (scenes/gen_spheres.py)
        import importlib.util
        spec = importlib.util.spec_from_file_location("g", os.path.join(sc, "gen_spheres.py"))
        g = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(g)
        return rtgo.Scene.from_json_text(g.dumps(g.generate(10000)))
    return rtgo.Scene.load_from_file(path)


for name, path, w, h, spp in cases:
    ctx = rtgo.Context(0)
    ctx.set_scene(load(path))
    st = rtgo.default_settings()
    st.samples = spp
    lin = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    rgba = torch.zeros(w * h * 4, dtype=torch.uint8, device="cuda")
    c = ctx.count(w, h, st, lin.data_ptr(), rgba.data_ptr())
    cam = c["camera_rays"]
    print(name, {k: v for k, v in c.items()})
    print("   per camera ray:", {k: round(v / cam, 3) for k, v in c.items()})
    print("   per shade event:", {k: round(v / max(1, c["shade_events"]), 2) for k, v in c.items()})
    ctx.close()
