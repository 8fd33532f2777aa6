#!/usr/bin/env python3
"""Frames in flight (dev tool): K headline frames rendered through F
contexts on F streams, frame i on context i % F, so a frame's low-occupancy
tail can overlap the next frame's start.  Prints the wall
time per frame for F = 1, 2, 3, 4 and checks that every context's image
equals the one-stream image."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd")]
import torch  # noqa: E402

import rtgo  # noqa: E402

W, H, SPP, K = 800, 600, 100, 40
scene = rtgo.Scene.load_from_file(os.path.join(ROOT, "scenes", "sphere_reflections_light_facing.json"))
st = rtgo.default_settings()
st.samples = SPP
ref = None
for F in (1, 2, 3, 4):
    ctxs, streams, bufs = [], [], []
    for _ in range(F):
        c = rtgo.Context(0)
        c.set_scene(scene)
        ctxs.append(c)
        streams.append(torch.cuda.Stream())
        bufs.append((torch.zeros(W * H * 3, dtype=torch.float32, device="cuda"),
                     torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda")))
    for i in range(2 * F):  # warm-up: builds every context's schedule
        j = i % F
        ctxs[j].render_async(W, H, st, bufs[j][0].data_ptr(), bufs[j][1].data_ptr(), streams[j].cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        j = i % F
        ctxs[j].render_async(W, H, st, bufs[j][0].data_ptr(), bufs[j][1].data_ptr(), streams[j].cuda_stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K * 1e3
    imgs = [b[0].cpu().numpy().tobytes() for b in bufs]
    if ref is None:
        ref = imgs[0]
    same = all(im == ref for im in imgs)
    print(f"frames in flight {F}: {dt:.4f} ms per frame, {W * H * SPP / dt / 1e3:.0f} Mrays/s, images equal: {same}",
          flush=True)
    for c in ctxs:
        c.close()
