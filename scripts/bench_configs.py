#!/usr/bin/env python3
"""Kernel time and Mrays/s of every BASELINE.json GPU config on one MI355X
(the bench.py headline is C2; this covers the others as well).

  C2  sphere_reflections_light 800x600x100 (facing variant; + as committed)
  C3  final_silver_prism_purple_cube 1200x900x100 (facing variant)
  C4  10k procedural spheres (scenes/gen_spheres.py) 1920x1080x64 (BVH)
  C5  10k spheres 3840x2160x256, ONE rank's share of 8 (tiles t % 8 == 0,
      packed layout): the per-GPU work of the 8-GPU config

Each line: kernel ms (HIP events, median of the timed renders after warm-up
renders that also build the schedule), Mrays/s = primary samples / kernel
time.  usage: bench_configs.py [--reps N] [--only C4,...]
"""
import argparse
import importlib.util
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd")]
import torch  # noqa: E402

import rtgo  # noqa: E402
from rtgo import shard  # noqa: E402


def spheres10k():
    spec = importlib.util.spec_from_file_location("gen_spheres", os.path.join(ROOT, "scenes", "gen_spheres.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    return rtgo.Scene.from_json_text(g.dumps(g.generate(10000)))


def scene_file(name):
    return lambda: rtgo.Scene.load_from_file(os.path.join(ROOT, "scenes", name))


CONFIGS = [
    ("C2", "sphere_reflections_light_facing", scene_file("sphere_reflections_light_facing.json"), 800, 600, 100, 0, 1),
    ("C2-committed", "sphere_reflections_light (as committed: black)", scene_file("sphere_reflections_light.json"),
     800, 600, 100, 0, 1),
    ("C3", "final_silver_prism_purple_cube_facing", scene_file("final_silver_prism_purple_cube_facing.json"),
     1200, 900, 100, 0, 1),
    ("C4", "10k spheres", spheres10k, 1920, 1080, 64, 0, 1),
    ("C5-rank0of8", "10k spheres, rank 0 of 8", spheres10k, 3840, 2160, 256, 0, 8),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    keep = set(filter(None, a.only.split(",")))
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    for cid, desc, load, w, h, spp, rank, world in CONFIGS:
        if keep and cid not in keep:
            continue
        ctx = rtgo.Context(0)
        ctx.set_scene(load())
        st = rtgo.default_settings()
        st.samples = spp
        n = shard.max_local_tiles(w, h, world) * 1024 if world > 1 else w * h
        layout = rtgo.RT_LAYOUT_PACKED_TILES if world > 1 else rtgo.RT_LAYOUT_IMAGE
        lin = torch.zeros(n * 3, dtype=torch.float32, device="cuda")
        rgba = torch.zeros(n * 4, dtype=torch.uint8, device="cuda")
        ms = []
        for i in range(a.reps + 2):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            ctx.render_async(w, h, st, lin.data_ptr(), rgba.data_ptr(), s.cuda_stream, rank, world, layout)
            e1.record()
            torch.cuda.synchronize()
            if i >= 2:
                ms.append(e0.elapsed_time(e1))
        k = statistics.median(ms)
        tx_n, ty_n = (w + 31) // 32, (h + 31) // 32
        px = sum(min(32, w - 32 * (t % tx_n)) * min(32, h - 32 * (t // tx_n)) for t in range(rank, tx_n * ty_n, world))
        rays = px * spp
        print(json.dumps({"config": cid, "scene": desc, "width": w, "height": h, "spp": spp, "max_depth": 50,
                          "rank": rank, "world": world, "kernel_ms": round(k, 4), "min_ms": round(min(ms), 4),
                          "mrays_per_s": round(rays / (k / 1e3) / 1e6, 1)}), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
