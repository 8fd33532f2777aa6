#!/usr/bin/env python3
"""The bench workload alone (no counting variant, no second scene): K renders
of the facing scene at 800x600x100 on one GPU.  Run under rocprofv3 --pmc by
scripts/profile.sh so each PMC pass sees only render_kernel<false,true>."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd")]
import torch  # noqa: E402

import rtgo  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
W, H, SPP = 800, 600, 100
SCENE = os.environ.get("PMC_SCENE", "")  # "spheres10k": config C4's scene at PMC_SIZE (W,H,SPP)
if os.environ.get("PMC_SIZE"):
    W, H, SPP = (int(v) for v in os.environ["PMC_SIZE"].split(","))
st = rtgo.default_settings()
st.samples = SPP
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
ctx = rtgo.Context(0)
if SCENE == "spheres10k":
    import importlib.util
    spec = importlib.util.spec_from_file_location("g", os.path.join(ROOT, "scenes", "gen_spheres.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    ctx.set_scene(rtgo.Scene.from_json_text(g.dumps(g.generate(10000))))
elif SCENE == "committed":  # the as-committed headline scene: black blocks only (the epilogue's stores alone)
    ctx.set_scene(rtgo.Scene.load_from_file(os.path.join(ROOT, "scenes", "sphere_reflections_light.json")))
else:
    ctx.set_scene(rtgo.Scene.load_from_file(os.path.join(ROOT, "scenes", "sphere_reflections_light_facing.json")))
lin = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
rgba = torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda")
for _ in range(K):
    ctx.render_async(W, H, st, lin.data_ptr(), rgba.data_ptr(), s.cuda_stream)
torch.cuda.synchronize()
print("rendered", K, "frames; linear sum", float(lin.double().sum()))
