#!/usr/bin/env python3
"""What one rank of an N-GPU strong-scaled frame costs (dev probe, not the
bench contract): the balanced (or strided) partition of the headline frame
over N ranks, and each rank's share rendered ALONE on this GPU with F frames
in flight (own context, stream and buffers per slot), K frames each.

The N-GPU step cannot finish before its slowest rank, so
  predicted N-GPU Mrays/s = W*H*spp / max over ranks (ms per share)
(the RCCL gather of ~1/N of 7.7 MB per frame and the unpack kernel come on
top; they run on a separate stream, overlapped with the next frames).

usage: rank_share_probe.py [N ...] [--fif F ...] [--batch B ...] [--block-work X ...] [--steps K] [--strided]
(--batch: B frames per launch, rt_context_render_frames_async; F launches in flight;
--block-work: rt_tuning.block_work, 0 = the library's default)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("worlds", type=int, nargs="*", default=[2, 4, 8])
    ap.add_argument("--fif", type=int, nargs="*", default=[1, 2, 4, 8])
    ap.add_argument("--batch", type=int, nargs="*", default=[1])
    ap.add_argument("--block-work", type=float, nargs="*", default=[0.0])
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--strided", action="store_true")
    ap.add_argument("--scene", default="sphere_reflections_light_facing.json")
    ap.add_argument("--size", type=int, nargs=2, default=[800, 600])
    ap.add_argument("--spp", type=int, default=100)
    args = ap.parse_args()
    import torch

    import rtgo

    W, H = args.size
    scene = rtgo.Scene.load_from_file(os.path.join(ROOT, "scenes", args.scene))

    def settings(seed):
        st = rtgo.default_settings()
        st.samples, st.max_depth, st.seed = args.spp, 50, seed
        return st

    out = {"frame": f"{args.scene} {W}x{H}x{args.spp}", "results": []}
    for world in args.worlds:
        ctx = rtgo.Context(0)
        ctx.set_scene(scene)
        part = rtgo.Partition(W, H, world) if args.strided else ctx.balanced_partition(W, H, settings(1), world)
        ctx.close()
        for F, B, bw in [(F, B, bw) for F in args.fif for B in args.batch for bw in args.block_work]:
            if True:
                per_rank = []
                nb = part.packed_bytes
                launches = max(1, args.steps // B)
                for rank in range(world):
                    slots = []
                    for _ in range(F):
                        c = rtgo.Context(0)
                        c.set_tuning(rtgo.default_tuning(block_work=bw))
                        c.set_scene(scene)
                        c.set_partition(part)
                        buf = torch.zeros(B * nb, dtype=torch.uint8, device="cuda")
                        s = torch.cuda.Stream()
                        lp = [buf.data_ptr() + f * nb for f in range(B)]
                        rp = [p + part.rgba_offset for p in lp]
                        slots.append((c, lp, rp, s, buf))
                        c.render_frames_async(W, H, settings(1), list(range(1, B + 1)), lp, rp, s.cuda_stream, rank,
                                              world, rtgo.RT_LAYOUT_PACKED_TILES)
                    torch.cuda.synchronize()
                    st = settings(1)
                    t0 = time.perf_counter()
                    for i in range(launches):
                        c, lp, rp, s, _ = slots[i % F]
                        c.render_frames_async(W, H, st, [2 + i * B + f for f in range(B)], lp, rp, s.cuda_stream,
                                              rank, world, rtgo.RT_LAYOUT_PACKED_TILES)
                    torch.cuda.synchronize()
                    ms = (time.perf_counter() - t0) / (launches * B) * 1e3
                    k1 = slots[0][0].last_kernel_seconds() * 1e3
                    per_rank.append({"rank": rank, "tiles": part.local_tiles(rank), "est_work": round(part.work(rank)),
                                     "ms_per_frame": round(ms, 4), "last_launch_ms": round(k1, 4)})
                    for c, _, _, _, _ in slots:
                        c.close()
                worst = max(r["ms_per_frame"] for r in per_rank)
                res = {"world": world, "partition": "strided" if args.strided else "balanced", "fif": F, "batch": B,
                       "block_work": bw or "default",
                       "worst_ms": worst, "predicted_mrays": round(W * H * args.spp / worst / 1e3, 1),
                       "ranks": per_rank}
                out["results"].append(res)
                print(json.dumps(res), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "rank_share_probe.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
