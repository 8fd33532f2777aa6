#!/usr/bin/env python3
"""Latency of one bounce of a lone path (dev tool).

The headline launch ends with a few 50-bounce paths running alone on their
SIMDs, so its length is set by the latency of a bounce, not
by throughput.  This probe measures that latency directly: the camera sits
inside a hollow metal sphere (roughness 0, so every ray reflects forever),
with the headline scene's five spheres and two lights inside; W x 1 pixels,
one sample each, so exactly W paths of max_depth bounces run in one wave.
Per-bounce latency = slope of kernel time over max_depth.  Variants switch
soft shadows off, drop a light, or drop the inner spheres.

usage: latency_probe.py [W]   (W <= 64: one block)
"""
import copy
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd")]
import torch  # noqa: E402

import rtgo  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 1
base = json.load(open(os.path.join(ROOT, "scenes", "sphere_reflections_light_facing.json")))
shell = {"type": "sphere", "position": [0, 0, 0], "radius": 30.0,
         "material": {"type": "metal", "color": [0.9, 0.9, 0.9], "roughness": 0.0}}


def scene(inner=True, lights=2):
    s = copy.deepcopy(base)
    s["objects"] = ([shell] + s["objects"]) if inner else [shell]
    s["lights"] = s["lights"][:lights]
    return rtgo.Scene.from_json_text(json.dumps(s))


TUN = {k: int(v) for k, v in (kv.split("=") for kv in filter(None, os.environ.get("PROBE_TUNING", "").split(",")))}


def time_depth(sc, depth, soft=1, reps=9):
    ctx = rtgo.Context(0)
    if TUN:  # e.g. PROBE_TUNING=tail_helpers=1,tail_depth=1,tail_every=1: the path runs in a tail helper
        ctx.set_tuning(rtgo.default_tuning(**TUN))
    ctx.set_scene(sc)
    st = rtgo.default_settings()
    st.samples = 1
    st.max_depth = depth
    st.soft_shadows = soft
    lin = torch.zeros(W * 3, dtype=torch.float32, device="cuda")
    rgba = torch.zeros(W * 4, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    ms = []
    for i in range(reps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ctx.render_async(W, 1, st, lin.data_ptr(), rgba.data_ptr(), s.cuda_stream)
        e1.record()
        torch.cuda.synchronize()
        if i >= 2:
            ms.append(e0.elapsed_time(e1) * 1e3)
    ctx.close()
    return statistics.median(ms)


if os.environ.get("PROBE_SECTIONS"):  # with an RT_WG_TIMING build (RTGO_LIB): section clocks of the one block
    for name, sc, soft in [("2 lights, soft", scene(), 1), ("no lights", scene(lights=0), 1)]:
        ctx = rtgo.Context(0)
        ctx.set_scene(sc)
        st = rtgo.default_settings()
        st.samples, st.max_depth, st.soft_shadows = 1, 51, soft
        dbg = torch.zeros(4096 * 48, dtype=torch.int64, device="cuda")
        ctx.set_debug_buffer(dbg.data_ptr())
        lin = torch.zeros(W * 3, dtype=torch.float32, device="cuda")
        rgba = torch.zeros(W * 4, dtype=torch.uint8, device="cuda")
        for _ in range(3):
            dbg.zero_()
            ctx.render_async(W, 1, st, lin.data_ptr(), rgba.data_ptr(), torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
        d = dbg.cpu().numpy().reshape(-1, 48)
        d = d[(d[:, 0] != 0) & ((d[:, 22] != 0) | (d[:, 7] > 1))]  # the block that ran the path
        for r in d:
            it = max(int(r[7]), 1)
            print(f"W={W} {name:16s} wave {(r[2] - r[0]) / 100.0:7.1f} us, iters {it}, clocks/iter: hit {r[3] / it:6.0f}"
                  f" light {r[4] / it:6.0f} (cone+hard {r[8] / it:6.0f}, soft {r[5] / it:6.0f}) scatter {r[9] / it:6.0f}"
                  f" fill {r[6]:6.0f}", flush=True)
            nb = int(r[22])
            if nb:  # a lone path ran (solo_path): its section clocks per bounce (s_memtime: shader clocks)
                names = ["loop+closest hit", "hit record", "tries+light vecs+cones+hard", "soft rays",
                         "lighting terms", "scatter"]
                print(f"   solo_path, {nb} bounces, clocks per bounce: " +
                      ", ".join(f"{n} {r[16 + k] / nb:6.0f}" for k, n in enumerate(names)) +
                      f"; total {sum(r[16:22]) / nb:6.0f}", flush=True)
                sub = ["tries", "light vectors", "their shuffles", "cones+hard+ballots", "soft rays of tries 0-63",
                       "soft rays of tries 0-127", "lighting terms"]
                print("   cumulative clocks within a section (parallel-lights form): " +
                      ", ".join(f"{n} {r[24 + k] / nb:6.0f}" for k, n in enumerate(sub)), flush=True)
        ctx.close()
    sys.exit(0)

CASES = [("2 lights, soft", scene(), 1), ("2 lights, hard only", scene(), 0),
         ("1 light, soft", scene(lights=1), 1), ("shell only, 2 lights, soft", scene(False), 1),
         ("no lights", scene(lights=0), 1)]
if os.environ.get("PROBE_QUICK"):  # the first and the last case only
    CASES = [CASES[0], CASES[-1]]
for name, sc, soft in CASES:
    t1, t26, t51 = time_depth(sc, 1, soft), time_depth(sc, 26, soft), time_depth(sc, 51, soft)
    print(f"W={W} {name:28s} depth1 {t1:7.1f} us  depth51 {t51:7.1f} us  per bounce {(t51 - t1) / 50:6.2f} us"
          f"  (26: {(t26 - t1) / 25:6.2f})", flush=True)
