#!/usr/bin/env python3
"""Determinism check (dev tool): render a config twice with each path and
compare bytes; then wavefront vs megakernel."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtgo  # noqa: E402

spec = importlib.util.spec_from_file_location("g", os.path.join(ROOT, "scenes", "gen_spheres.py"))
g = importlib.util.module_from_spec(spec)
spec.loader.exec_module(g)
scene = rtgo.Scene.from_json_text(g.dumps(g.generate(10000)))
W, H = int(sys.argv[1]), int(sys.argv[2])
SPP = int(sys.argv[3]) if len(sys.argv) > 3 else 64


def render(mega):
    ctx = rtgo.Context(0)
    ctx.set_tuning(rtgo.default_tuning(path=rtgo.RT_PATH_MEGAKERNEL if mega else rtgo.RT_PATH_AUTO))
    ctx.set_scene(scene)
    st = rtgo.default_settings()
    st.samples, st.seed = SPP, 1
    lin = torch.full((W * H * 3,), float("nan"), dtype=torch.float32, device="cuda")
    rgba = torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda")
    ctx.render_async(W, H, st, lin.data_ptr(), rgba.data_ptr(), 0)
    torch.cuda.synchronize()
    ctx.close()
    return lin.cpu().numpy().reshape(H, W, 3)


wf = [render(False) for _ in range(3)]
mk = [render(True) for _ in range(1)] if not os.environ.get("NO_MK") else [None]
pairs = [("wf0 vs wf1", wf[0], wf[1]), ("wf0 vs wf2", wf[0], wf[2])]
if mk[0] is not None:
    pairs.append(("wf0 vs mk", wf[0], mk[0]))
tag = os.environ.get("TAG", "")
for name, a, b in pairs:
    bad = np.argwhere((a != b).any(axis=2))
    print(f"{tag} {W}x{H}x{SPP} {name}: {len(bad)} pixels differ", bad[:5].tolist(), flush=True)
    if len(bad):
        y, x = bad[0]
        print("   e.g.", a[y, x].tolist(), b[y, x].tolist())
