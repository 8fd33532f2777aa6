#!/usr/bin/env python3
"""C4 per-kernel frame times under wavefront tuning variants (dev probe, not
the bench contract): config C4's scene (10k spheres) at 1920x1080x64, depth
50, one frame per variant after a warm-up frame, with rt_context_profile's
per-kernel HIP-event times.  Variants: KEY=VAL[,KEY=VAL] of rt_tuning.

usage: c4_tuning_probe.py "wf_trav_block=1024" "wf_trav_block=768" ...
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd"), os.path.join(ROOT, "tests")]


def main():
    import torch

    import rtgo
    from bench import CONFIGS, load_scene

    spec, W, H, SPP = CONFIGS["c4"][:4]
    scene = load_scene(rtgo, spec)
    lin = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    set_env = []
    for var in sys.argv[1:] or [""]:
        over = {}
        for k in set_env:  # (a variant's environment switches end with it)
            os.environ.pop(k, None)
        set_env = []
        for kv in filter(None, var.split(",")):
            k, _, v = kv.partition("=")
            if k.startswith("env."):  # an environment switch of the library (env.RTGO_BVH4=0)
                os.environ[k[4:]] = v
                set_env.append(k[4:])
                continue
            over[k] = float(v) if "." in v else int(v)
        ctx = rtgo.Context(0)
        ctx.set_tuning(rtgo.default_tuning(**over))
        ctx.set_scene(scene)
        st = rtgo.default_settings()
        st.samples = SPP
        ctx.render_async(W, H, st, lin.data_ptr(), 0)
        torch.cuda.synchronize()
        ctx.profile(True)
        t0 = time.perf_counter()
        st.seed = 2
        ctx.render_async(W, H, st, lin.data_ptr(), 0)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        ks = ctx.kernel_seconds()
        row = {"variant": var, "frame_ms": round(wall * 1e3, 2),
               "kernel_ms": {k: round(v[0] * 1e3, 2) for k, v in ks.items()},
               "checksum": float(lin.double().sum())}
        if os.environ.get("PROBE_COUNT"):  # one counted frame: the soft-shadow stage's own counts
            c = ctx.count(W, H, st, lin.data_ptr(), 0, full=True)
            row["counts"] = c.as_dict()
            row["soft_stage_counts"] = c.soft_occlusion_dict()
        ctx.close()
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
