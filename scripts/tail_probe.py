#!/usr/bin/env python3
"""Tail helpers by tuning (dev tool): the headline frame
rendered one at a time and K frames per launch, kernel ms (HIP events) and
paths exported per frame, for each rt_tuning.tail_* setting given.

usage: tail_probe.py [SPEC ...]   SPEC = "name:key=val,key=val" (e.g.
       "off:tail_helpers=-1" "d8:tail_depth=8"); default: a small sweep
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd")]
import torch  # noqa: E402

import rtgo  # noqa: E402

W, H = 800, 600
K = int(os.environ.get("TAIL_K", "20"))
REPS = int(os.environ.get("TAIL_REPS", "15"))


def parse(spec):
    name, _, kv = spec.partition(":")
    tun = {}
    for item in filter(None, kv.split(",")):
        k, _, v = item.partition("=")
        tun[k] = int(v)
    return name, tun


def run(scene, tun):
    ctx = rtgo.Context(0)
    ctx.set_tuning(rtgo.default_tuning(**tun))
    ctx.set_scene(scene)
    st = rtgo.default_settings()
    lin = torch.zeros((K, W * H * 3), dtype=torch.float32, device="cuda")
    rgba = torch.zeros((K, W * H * 4), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    one = []
    e0 = ctx.stats()["tail_exported"]
    for i in range(REPS + 2):
        st.seed = 100 + i
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        ctx.render_async(W, H, st, lin[0].data_ptr(), rgba[0].data_ptr(), s.cuda_stream)
        b.record()
        torch.cuda.synchronize()
        if i >= 2:
            one.append(a.elapsed_time(b))
    e1 = ctx.stats()["tail_exported"]
    st.seed = 1
    bat = []
    for r in range(4):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        ctx.render_frames_async(W, H, st, [1000 + 100 * r + f for f in range(K)], [lin[f].data_ptr() for f in range(K)],
                                [rgba[f].data_ptr() for f in range(K)], s.cuda_stream)
        b.record()
        torch.cuda.synchronize()
        if r >= 1:
            bat.append(a.elapsed_time(b) / K)
    e2 = ctx.stats()
    dbg = ctx.tail_debug()
    ctx.close()
    return {"one_frame_ms": round(statistics.median(one), 4), "one_frame_min": round(min(one), 4),
            "exported_per_frame": round((e1 - e0) / (REPS + 2), 1),
            "batched_ms_per_frame": round(statistics.median(bat), 4),
            "exported_per_batched_frame": round((e2["tail_exported"] - e1) / (4 * K), 1),
            "errors": e2["tail_errors"], "debug": dbg,
            "us_per_path_solo": round(dbg["solo_ticks"] / max(1, dbg["paths_done"]) / 100, 2),
            "us_per_export": round(dbg["export_ticks"] / max(1, dbg["exported"]) / 100, 2)}


def main():
    specs = sys.argv[1:] or ["off:tail_helpers=-1", "default:", "d4:tail_depth=4", "d8:tail_depth=8",
                             "k1:tail_paths=1", "k2d4:tail_paths=2,tail_depth=4", "h64:tail_helpers=64"]
    name = os.environ.get("TAIL_SCENE", "sphere_reflections_light_facing.json")  # (W, H: the headline's)
    scene = rtgo.Scene.load_from_file(os.path.join(ROOT, "scenes", name))
    for spec in specs:
        name, tun = parse(spec)
        print(json.dumps({"name": name, "tuning": tun, **run(scene, tun)}), flush=True)


if __name__ == "__main__":
    main()
