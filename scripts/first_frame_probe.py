#!/usr/bin/env python3
"""Where a first frame's time goes (dev tool): fresh contexts rendering the
headline frame with a new schedule (pilot render + GPU block building), per
pilot variant: wall clock of the first frame, its render kernel, and the
render kernel of the same context's next frames (cached schedule).
usage: first_frame_probe.py [reps]"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd")]
import torch  # noqa: E402

import rtgo  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
scene_name = sys.argv[2] if len(sys.argv) > 2 else "sphere_reflections_light_facing.json"
W, H = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (800, 600)
scene = rtgo.Scene.load_from_file(os.path.join(ROOT, "scenes", scene_name))
lin = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
rgba = torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda")
s = torch.cuda.Stream()
VARIANTS = [("pilot full depth", dict(pilot=1)), ("pilot depth 8", dict(pilot=1, pilot_depth=8)),
            ("pilot depth 12", dict(pilot=1, pilot_depth=12)), ("pilot depth 16", dict(pilot=1, pilot_depth=16)),
            ("pilot depth 24", dict(pilot=1, pilot_depth=24)), ("no pilot", dict(pilot=0))]
for i in range(2):  # warm-up: code objects, allocator
    ctx = rtgo.Context(0)
    ctx.set_scene(scene)
    ctx.render_async(W, H, rtgo.default_settings(), lin.data_ptr(), rgba.data_ptr(), s.cuda_stream)
    s.synchronize()
    ctx.close()
for name, tun in VARIANTS:
    first, fk, ck = [], [], []
    for i in range(reps):
        st = rtgo.default_settings()
        st.seed = 1 + i
        ctx = rtgo.Context(0)
        ctx.set_tuning(rtgo.default_tuning(**tun))
        ctx.set_scene(scene)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ctx.render_async(W, H, st, lin.data_ptr(), rgba.data_ptr(), s.cuda_stream)
        s.synchronize()
        first.append(time.perf_counter() - t1)
        fk.append(ctx.last_kernel_seconds())
        for j in range(4):  # the same key again: cached schedule
            st.seed = 100 + j
            ctx.render_async(W, H, st, lin.data_ptr(), rgba.data_ptr(), s.cuda_stream)
            s.synchronize()
            ck.append(ctx.last_kernel_seconds())
        ctx.close()
    m = lambda v: 1e3 * statistics.median(v)  # noqa: E731
    print(f"{name:18s} first frame {m(first):.3f} ms (its render kernel {m(fk):.3f}) | cached kernel "
          f"{m(ck):.3f} ms", flush=True)
