#!/usr/bin/env python3
"""Do two C4 frames overlap on one GPU? (dev probe, not the bench contract)

A BVH frame's wavefront loop is host-driven and returns when the frame is
done, so frames in flight need one host thread each.  Times N frames one at
a time, then the same N frames from two threads (own context and stream
each): the ratio bounds what overlapping two path pools inside one frame
could gain (their launches' drains filled by the other pool's work)."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import rtgo  # noqa: E402
from scene_cases import spheres10k_scene  # noqa: E402

W, H, SPP = 1920, 1080, int(os.environ.get("SPP", "64"))
N = int(os.environ.get("FRAMES", "4"))
scene = spheres10k_scene(rtgo)
ctxs, bufs, streams = [], [], []
for k in range(2):
    c = rtgo.Context(0)
    c.set_scene(scene)
    ctxs.append(c)
    bufs.append((torch.zeros(W * H * 3, dtype=torch.float32, device="cuda"),
                 torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda")))
    streams.append(torch.cuda.Stream())


def frame(k, seed):
    st = rtgo.default_settings()
    st.samples, st.seed = SPP, seed
    lin, rgba = bufs[k]
    ctxs[k].render_async(W, H, st, lin.data_ptr(), rgba.data_ptr(), streams[k].cuda_stream)
    streams[k].synchronize()


for k in range(2):
    frame(k, 1)  # set-up (buffers, BVH upload)
t0 = time.perf_counter()
for i in range(N):
    frame(0, 10 + i)
one = (time.perf_counter() - t0) / N


def worker(k):
    for i in range(k, N, 2):
        frame(k, 10 + i)


t0 = time.perf_counter()
ths = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
for t in ths:
    t.start()
for t in ths:
    t.join()
two = (time.perf_counter() - t0) / N
print(f"C4-size frame {W}x{H}x{SPP}: one at a time {one * 1e3:.1f} ms per frame, "
      f"two threads {two * 1e3:.1f} ms per frame ({one / two:.3f}x)")
