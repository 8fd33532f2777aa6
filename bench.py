#!/usr/bin/env python3
"""Benchmark: Mrays/s of the gfx950 renderer on BASELINE.json's config.

metric  : Mrays/s = W*H*spp / render time (primary samples per second, the
          reference's published rays_per_second semantics, README.md:61,
          demo-assets/sphere_reflections_light_benchmark.json:12).
workload: configs[1]: sphere_reflections_light, 800x600, 100 spp, depth 50,
          soft shadows + recursive reflections, 1 GPU.  The committed scene
          puts every object behind the reference's fixed -Z camera
          (renderer.go:377-390), so its faithful render is black.  The
          headline `value` is therefore the "facing" variant (camera z=+8,
          scenes/sphere_reflections_light_facing.json: same objects, lights and
          materials), which is MORE work.  --with-as-committed also times
          the as-committed scene ("as_committed" in the output).
step    : one render of the frame with the scene and output buffers resident
          in HBM.  Frames are rendered with F frames in flight
          (--frames-in-flight, default 2): step i runs on context/stream
          i % F with its own output buffers, so a frame's low-occupancy tail
          (its last few 50-bounce paths) overlaps the next
          frame's start.  Every step still renders one whole frame; `value`
          is whole-job throughput over the K steps.  The same K frames are
          also timed one at a time (F = 1, the reference's synchronous
          Render): "one_frame_in_flight" reports that rate and the frame
          latency.  For N>1 a step also includes the RCCL gather of the packed
          tiles to rank 0 and the unpack kernel there.  Like the scene
          upload, the work schedule of a (scene, frame, settings) key is
          built by the first frame (one-sample pilot render + host block
          building) and reused; "first_frame_ms" times a
          frame on a fresh context that builds it.
scaling : weak.  At N GPUs the frame is 800 x (600*N): the same viewport at
          N-fold vertical sample density.  Its 32x32 tiles are dealt
          t -> t % N, so every GPU traces about one
          800x600x100 frame of primary samples.  value = all ranks' samples /
          max-over-ranks time.

usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--scene PATH]
                       [--width 800 --height 600 --spp 100 --depth 50]
                       [--no-cpu-baseline] [--strong]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "concurrent-raytracer-go_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

# FP64 operations per counted event: the adds, muls,
# divides and square roots of the reference's formulas, 1 each.
FLOPS_PER_EVENT = {
    "camera_rays": 12,     # u, v (2 add + 2 div) + getRay (8)
    "sphere_tests": 20,    # Sphere.Hit up to the discriminant test (+ avg root work)
    "triangle_tests": 46,  # Moller-Trumbore to the t test
    "box_tests": 12,       # slab test: 6 sub + 6 mul
    "shade_events": 75,    # hit record + scatter + path update
    "light_evals": 60,     # direct-lighting terms per light
    "shadow_rays": 15,     # soft direction: scale, add, normalize
    "rng_draws": 5,        # unit conversion + rejection arithmetic
}
PEAK_FP64_TFLOPS = 78.6   # MI355X FP64 vector (= FP64 matrix) peak: 256 CU x 2.4 GHz x 128 FLOP/clk
PEAK_HBM_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
PMC_FILE = os.path.join(ROOT, "profiles", "r01_pmc_traffic.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)  # 100 frames: 40 ms; fewer steps weigh the un-overlapped first start and last tail (20: -6 %)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "sphere_reflections_light_facing.json"))
    ap.add_argument("--as-committed", default=os.path.join(ROOT, "scenes", "sphere_reflections_light.json"))
    ap.add_argument("--width", type=int, default=800)
    ap.add_argument("--height", type=int, default=600)
    ap.add_argument("--spp", type=int, default=100)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--strong", action="store_true", help="fixed 800x600 frame for every N (strong scaling)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--with-as-committed", action="store_true",
                    help="also time the as-committed (black) scene; off by default so the profiled command's "
                         "render_kernel launches are all of the headline workload")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--frames-in-flight", type=int, default=2,
                    help="frames rendered concurrently (own context, stream and buffers each)")
    return ap.parse_args()


class Frame:
    """Device buffers and one render step of this rank."""

    def __init__(self, rtgo, torch, dist, ctx, w, h, st, rank, world, device, stream=None):
        self.stream = stream
        self.rtgo, self.torch, self.dist = rtgo, torch, dist
        self.ctx, self.w, self.h, self.st = ctx, w, h, st
        self.rank, self.world = rank, world
        dev = torch.device("cuda", device)
        if world == 1:
            self.layout = rtgo.RT_LAYOUT_IMAGE
            n = w * h
        else:
            from rtgo import shard

            self.layout = rtgo.RT_LAYOUT_PACKED_TILES
            self.max_local = shard.max_local_tiles(w, h, world)  # rank 0 owns the most tiles
            n = self.max_local * 1024
            if rank == 0:
                self.g_lin = torch.empty(world * n * 3, dtype=torch.float32, device=dev)
                self.g_rgba = torch.empty(world * n * 4, dtype=torch.uint8, device=dev)
                self.img_lin = torch.zeros(w * h * 3, dtype=torch.float32, device=dev)
                self.img_rgba = torch.zeros(w * h * 4, dtype=torch.uint8, device=dev)
        self.lin = torch.zeros(n * 3, dtype=torch.float32, device=dev)
        self.rgba = torch.zeros(n * 4, dtype=torch.uint8, device=dev)

    def render(self, stream):
        self.ctx.render_async(self.w, self.h, self.st, self.lin.data_ptr(), self.rgba.data_ptr(), stream,
                              self.rank, self.world, self.layout)

    def gather(self, stream):
        """The one collective (rtgo.shard.gather_packed: an equal-size
        gather of the packed tiles to rank 0 over RCCL), then the unpack
        kernel on rank 0."""
        if self.world == 1:
            return
        from rtgo import shard

        shard.gather_packed(self.dist, self.lin, self.world, self.rank, getattr(self, "g_lin", None))
        shard.gather_packed(self.dist, self.rgba, self.world, self.rank, getattr(self, "g_rgba", None))
        if self.rank == 0:
            self.rtgo.unpack_tiles_async(self.w, self.h, self.world, self.max_local, self.g_lin.data_ptr(),
                                         self.g_rgba.data_ptr(), self.img_lin.data_ptr(),
                                         self.img_rgba.data_ptr(), stream)

    def counts(self, stream):
        return self.ctx.count(self.w, self.h, self.st, self.lin.data_ptr(), self.rgba.data_ptr(), stream,
                              self.rank, self.world, self.layout)


def time_steps(frames, torch, dist, world, steps, warmup):
    """W untimed steps, then K timed steps between barrier + synchronize on
    both sides; step i renders frames[i % F] on its own stream (F frames in
    flight); returns (max-over-ranks seconds, per-launch kernel ms).  Kernel
    durations come from HIP events recorded on the stream each kernel is
    launched on."""
    F = len(frames)
    for i in range(warmup):
        fr = frames[i % F]
        with torch.cuda.stream(fr.stream):
            fr.render(fr.stream.cuda_stream)
            fr.gather(fr.stream.cuda_stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = []
    t0 = time.perf_counter()
    for i in range(steps):
        fr = frames[i % F]
        with torch.cuda.stream(fr.stream):  # events and the gather's stream: this frame's
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            fr.render(fr.stream.cuda_stream)
            e1.record()
            evs.append((e0, e1))
            fr.gather(fr.stream.cuda_stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, [a.elapsed_time(b) for a, b in evs]


def first_frame_ms(rtgo, torch, dist, args, W, H, st, rank, world, local, stream_ptr):
    """One frame on a fresh context, including what the timed steps reuse:
    the per-(scene, frame, settings) schedule (frustum masks, the one-sample
    pilot render, block building and upload).  Wall clock,
    max over ranks."""
    ctx = rtgo.Context(local)
    ctx.set_scene(rtgo.Scene.load_from_file(args.scene))
    frame = Frame(rtgo, torch, dist, ctx, W, H, st, rank, world, local, torch.cuda.current_stream())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    frame.render(stream_ptr)
    frame.gather(stream_ptr)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    if world > 1:
        t = torch.tensor([ms], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
    ctx.close()
    return ms


def flops_of(counts):
    return sum(FLOPS_PER_EVENT[k] * counts.get(k, 0) for k in FLOPS_PER_EVENT)


def cpu_baseline(args, rtgo, st):
    """The oracle (C restatement of the Go goroutine path) on the host cores.
    Bounded sample: the full 800x600x100 frame when it is cheap (the facing
    scene is mostly sky: ~1.5 s on 8 cores), median of 3 after a warm-up."""
    import oracle

    scene = rtgo.Scene.load_from_file(args.scene)
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    threads = args.cpu_threads or min(16, cores)
    oracle.render(scene, args.width, args.height, st, nthreads=threads, max_tiles=16)  # warm-up
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        oracle.render(scene, args.width, args.height, st, nthreads=threads)
        times.append(time.perf_counter() - t0)
    times.sort()
    secs = times[1]
    rays = args.width * args.height * args.spp
    return {
        "value": round(rays / secs / 1e6, 3),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "sample": f"full {args.width}x{args.height}x{args.spp}spp frame of the facing scene, median of 3 runs "
                  f"({secs:.2f} s) after 1 warm-up; oracle/oracle.c on {threads} threads (tile queue of "
                  f"renderer.go:67-148; the Go toolchain is absent, SURVEY.md §8c)",
    }


def pmc_traffic(workload):
    """HBM bytes per launch from the committed rocprofv3 PMC passes
    (profiles/r01_pmc_traffic.json, made by scripts/pmc_traffic.py with the
    gfx950 corrections of MI355X_MICROARCH.md §HBM), if they match."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("workload") != workload:
        return None
    return d.get("hbm_bytes_per_launch")


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import rtgo

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"--gpus {args.gpus} needs torch.distributed.run with {args.gpus} processes (WORLD_SIZE={world})",
              file=sys.stderr)
        sys.exit(2)
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    W = args.width
    H = args.height if args.strong else args.height * world  # weak scaling: N-fold vertical sample density
    st = rtgo.default_settings()
    st.samples, st.max_depth, st.seed = args.spp, args.depth, args.seed
    st.num_workers = world
    # a dedicated stream: render kernel, timing events and gather all run on
    # it (torch.cuda.Event records on the current stream)
    bench_stream = torch.cuda.Stream()
    torch.cuda.set_stream(bench_stream)
    stream_ptr = bench_stream.cuda_stream

    F = max(1, args.frames_in_flight)
    scene = rtgo.Scene.load_from_file(args.scene)
    frames = []
    for j in range(F):  # F frames in flight: own context (schedule), stream and buffers each
        ctx = rtgo.Context(local)
        ctx.set_scene(scene)
        fr = Frame(rtgo, torch, dist, ctx, W, H, st, rank, world, local,
                   bench_stream if j == 0 else torch.cuda.Stream())
        with torch.cuda.stream(fr.stream):  # set-up: builds this context's schedule (like the scene upload)
            fr.render(fr.stream.cuda_stream)
            fr.gather(fr.stream.cuda_stream)
        frames.append(fr)
    counts = frames[0].counts(stream_ptr)  # algorithmic work of this rank's launch (counting variant, untimed)
    torch.cuda.synchronize()
    elapsed, kms = time_steps(frames, torch, dist, world, args.steps, args.warmup)
    # the same frames one at a time (the reference's synchronous Render)
    elapsed1, kms1 = time_steps(frames[:1], torch, dist, world, args.steps, args.warmup) if F > 1 else (elapsed, kms)
    first_ms = first_frame_ms(rtgo, torch, dist, args, W, H, st, rank, world, local, stream_ptr)

    as_committed = None
    if args.with_as_committed:
        ctx2 = rtgo.Context(local)
        ctx2.set_scene(rtgo.Scene.load_from_file(args.as_committed))
        frame2 = Frame(rtgo, torch, dist, ctx2, W, H, st, rank, world, local, bench_stream)
        elapsed2, kms2 = time_steps([frame2], torch, dist, world, args.steps, args.warmup)
        as_committed = {
            "scene": "sphere_reflections_light.json as committed (renders black: objects behind the camera)",
            "value": round(W * H * args.spp * args.steps / elapsed2 / 1e6, 3),
            "ms_per_step": round(elapsed2 / args.steps * 1e3, 4),
            "kernel_ms": round(sum(kms2) / len(kms2), 4),
        }

    rays = W * H * args.spp  # all ranks together
    value = rays * args.steps / elapsed / 1e6
    kernel_s = sum(kms) / len(kms) / 1e3  # this rank's average launch
    flops = flops_of(counts)
    achieved_tf = flops / kernel_s / 1e12
    npix_local = rtgo.tiles_for_rank(W, H, rank, world) * 1024 if world > 1 else W * H
    # algorithmic HBM bytes: framebuffer write (float3 + RGBA8 = 16 B/pixel)
    # + the flattened scene read once per workgroup-resident copy (<= 4 KB)
    hbm_bytes = npix_local * 16 + 4096
    achieved_gbs = hbm_bytes / kernel_s / 1e9
    workload = "sphere_reflections_light_facing %dx%d %dspp depth %d" % (W, H, args.spp, args.depth)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, rtgo, st)

    if rank == 0:
        out = {
            "metric": "Mrays/sec at 800x600x100spp max_depth=50 (sphere_reflections_light)",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            # a first frame also builds the schedule that steps reuse (pilot render + host blocks)
            "first_frame_ms": round(first_ms, 4),
            "frames_in_flight": F,
            "one_frame_in_flight": {
                "value": round(rays * args.steps / elapsed1 / 1e6, 3),
                "ms_per_step": round(elapsed1 / args.steps * 1e3, 4),
                "kernel_ms": round(sum(kms1) / len(kms1), 4),
            },
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,  # BASELINE.md has no published number on this hardware/config
            "dtype": "f64",
            "data": "synthetic: the reference's scene JSON (camera facing the objects), seeded counter-keyed "
                    "RNG (seed %d)" % args.seed,
            "config": {
                "workload": workload + ", soft shadows, recursive reflections",
                "width": W, "height": H, "spp": args.spp, "max_depth": args.depth,
                "parallelism": "tiles t%%%d + RCCL gather" % world if world > 1 else "1 GPU",
                "frames_in_flight": F,
            },
            "roofline": {
                "bound": "valu",
                "achieved": round(achieved_tf, 4),
                "peak": PEAK_FP64_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved_tf / PEAK_FP64_TFLOPS, 5),
                "traffic": pmc_traffic(workload),
                "kernel": "rtgo::render_kernel<false, true, false>",
                "kernel_ms": round(kernel_s * 1e3, 4),
                "flops_per_launch": flops,
                "note": "FP64 VALU-bound branchy path (binary64 like the Go reference; no matrix shape, no MFMA). "
                        "achieved = algorithmic FP64 ops of one launch (the kernel's own event counts x "
                        "DESIGN.md per-event costs) / average launch time (HIP events on the stream each launch runs on; "
                        "with frames in flight a launch shares the GPU with its neighbours' tails). "
                        "traffic = HBM bytes per launch from rocprofv3 FETCH_SIZE+WRITE_SIZE passes.",
            },
            "roofline_hbm": {
                "bound": "hbm",
                "achieved": round(achieved_gbs, 3),
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / PEAK_HBM_GBS, 7),
                "algorithmic_bytes_per_launch": hbm_bytes,
            },
            "counts_rank0": counts,
            "as_committed": as_committed,
            "cpu_baseline": cpu,
        }
        if cpu:
            out["gpu_over_cpu"] = round(value / cpu["value"], 1)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
