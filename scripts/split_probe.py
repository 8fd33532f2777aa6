#!/usr/bin/env python3
"""Schedule shape of the headline frame (dev probe): work blocks and split
pixels of the one-frame schedule and of a batched launch's, and the bytes of
the split pixels' per-sample radiance rows (24 B per sample, written and read
back once per frame) against the PMC traffic of profiles/r05_pmc_traffic.json.

usage: split_probe.py [config]   (default c2)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd")]


def main():
    import torch

    import rtgo
    from bench import CONFIGS, load_scene

    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    spec, W, H, SPP = CONFIGS[cfg][:4]
    scene = load_scene(rtgo, spec)
    out = {"config": cfg}
    for label, nframes in (("one_frame", 1), ("batched_10", 10)):
        ctx = rtgo.Context(0)
        ctx.set_scene(scene)
        st = rtgo.default_settings()
        st.samples = SPP
        lins = [torch.zeros(W * H * 3, dtype=torch.float32, device="cuda") for _ in range(nframes)]
        if nframes == 1:
            ctx.render_async(W, H, st, lins[0].data_ptr(), 0)
        else:
            ctx.render_frames_async(W, H, st, list(range(1, nframes + 1)), [t.data_ptr() for t in lins])
        torch.cuda.synchronize()
        s = ctx.stats()
        rows = s["split_pixels"] * SPP * 3 * 8
        out[label] = {"blocks": s["blocks"], "split_pixels": s["split_pixels"],
                      "split_row_bytes_per_frame": rows,
                      "note": "each split pixel's samples are stored (24 B each) and summed in sample order"}
        ctx.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
