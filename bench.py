#!/usr/bin/env python3
"""Benchmark: Mrays/s of the gfx950 renderer on BASELINE.json's configs.

metric  : Mrays/s = W*H*spp / render time (primary samples per second, the
          reference's published rays_per_second semantics, README.md:61,
          demo-assets/sphere_reflections_light_benchmark.json:12).
workload: --config c2 (default, the headline): BASELINE configs[1],
          sphere_reflections_light 800x600x100 spp, depth 50, soft shadows +
          recursive reflections.  The committed scene puts every object
          behind the reference's fixed -Z camera (renderer.go:377-390), so
          its faithful render is black; the headline uses the "facing"
          variant (camera z = +8, same objects, lights, materials), which is
          MORE work.  Other configs: c2_committed (black), c3 (silver prism
          scene facing, 1200x900x100), c4 (10k procedural spheres, BVH,
          1920x1080x64), c5 (10k spheres 3840x2160x256: the 8-GPU config).
step    : one render of a whole frame with the scene and output buffers
          resident in HBM; every step renders a DIFFERENT image (seed + i).
          Frames are rendered with F frames in flight (--frames-in-flight,
          default 2 for c2/c3): step i runs on context/stream i % F with its
          own buffers, so a frame's low-occupancy tail (its last 50-bounce
          paths) overlaps the next frame's start.  The same
          frames are also timed one at a time (the reference's synchronous
          Render): "one_frame_in_flight".  For N>1 a step also includes the
          one RCCL gather of the ranks' packed shares to rank 0
          (rt_comm_gather_tiles_async: librtgo's own ncclSend/ncclRecv over
          xGMI) and the unpack kernel there.  The work schedule of a (scene,
          frame, settings) key is built by the first frame and reused
          (seeds excluded from the key).
end to end: "render_e2e" (N=1): the blocking Render of the C ABI
          (rt_renderer_render: scene check + upload, schedule, kernels,
          device->host copy of the image), median of 7 calls with distinct
          seeds on one renderer object (NewParallelRenderer once, Render per
          frame, as cmd/raytracer uses it); "oneshot" = rt_render, which also
          creates and destroys the device contexts every call.
scaling : c2 weak by default: at N GPUs the frame is 800 x (600*N) (per-GPU
          work fixed at one 800x600x100 frame of samples); --strong keeps
          800x600.  c4 / c5: strong (the frame is fixed).  Tiles are dealt
          t -> t % N.  value = all ranks' samples /
          max-over-ranks time.

usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c2_committed|c3|c4|c5]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "concurrent-raytracer-go_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

# FP64 operations per counted event: the adds, muls,
# divides and square roots of the reference's formulas, 1 each, for the
# work the kernel EXECUTES (primitives culled as provably missed are neither
# executed nor counted).
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
PMC_FILE = os.path.join(ROOT, "profiles", "r02_pmc_traffic.json")

CONFIGS = {
    # name: (scene, W, H, spp, label, default steps, default frames in flight)
    "c2": ("sphere_reflections_light_facing.json", 800, 600, 100, "sphere_reflections_light_facing", 100, 2),
    "c2_committed": ("sphere_reflections_light.json", 800, 600, 100,
                     "sphere_reflections_light as committed (black: objects behind the -Z camera)", 100, 2),
    "c3": ("final_silver_prism_purple_cube_facing.json", 1200, 900, 100, "final_silver_prism_purple_cube_facing",
           50, 2),
    "c4": ("gen:10000", 1920, 1080, 64, "procedural 10k spheres (scenes/gen_spheres.py, BVH)", 3, 1),
    "c5": ("gen:10000", 3840, 2160, 256, "procedural 10k spheres (scenes/gen_spheres.py, BVH)", 1, 1),
}
KERNELS = {  # the dominant kernel of each config (rocprofv3 --stats, profiles/)
    "c2": "rtgo::render_kernel<false, true, false, false>",
    "c2_committed": "rtgo::render_kernel<false, true, false, false>",
    "c3": "rtgo::render_kernel<false, true, false, false>",
    "c4": "wavefront bounce loop (wf_occlude<false, true, true> dominant)",
    "c5": "wavefront bounce loop (wf_occlude<false, true, true> dominant)",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=0, help="timed steps (default per config: c2 100)")
    ap.add_argument("--warmup", type=int, default=-1, help="untimed steps (default: c2/c3 3, c4/c5 1)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--spp", type=int, default=0, help="override the config's spp")
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--strong", action="store_true", help="c2: fixed 800x600 frame for every N (strong scaling)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--frames-in-flight", type=int, default=0,
                    help="frames rendered concurrently (own context, stream and buffers each)")
    return ap.parse_args()


def load_scene(rtgo, spec):
    if spec.startswith("gen:"):
        from scene_cases import spheres10k_scene

        return spheres10k_scene(rtgo, int(spec[4:]))
    return rtgo.Scene.load_from_file(os.path.join(ROOT, "scenes", spec))


class Frame:
    """Device buffers and one render step of this rank.

    world 1: the W*H image.  world > 1: this rank's packed share
    (rt_packed_bytes: float3 + RGBA8 per pixel of its tiles); rank 0 renders
    its share in place into the gather buffer and unpacks the image there."""

    def __init__(self, rtgo, torch, ctx, w, h, rank, world, device, stream, comm):
        self.rtgo, self.ctx, self.w, self.h = rtgo, ctx, w, h
        self.rank, self.world, self.stream, self.comm = rank, world, stream, comm
        dev = torch.device("cuda", device)
        if world == 1:
            self.layout = rtgo.RT_LAYOUT_IMAGE
            self.lin = torch.zeros(w * h * 3, dtype=torch.float32, device=dev)
            self.rgba = torch.zeros(w * h * 4, dtype=torch.uint8, device=dev)
            self.p_lin, self.p_rgba = self.lin.data_ptr(), self.rgba.data_ptr()
            return
        self.layout = rtgo.RT_LAYOUT_PACKED_TILES
        nb = rtgo.packed_bytes(w, h, world)
        if rank == 0:
            self.gathered = torch.zeros(world * nb, dtype=torch.uint8, device=dev)
            self.share = self.gathered[:nb]
            self.img_lin = torch.zeros(w * h * 3, dtype=torch.float32, device=dev)
            self.img_rgba = torch.zeros(w * h * 4, dtype=torch.uint8, device=dev)
        else:
            self.gathered = None
            self.share = torch.zeros(nb, dtype=torch.uint8, device=dev)
        self.p_lin = self.share.data_ptr()
        self.p_rgba = self.share.data_ptr() + rtgo.packed_rgba_offset(w, h, world)

    def render(self, st):
        self.ctx.render_async(self.w, self.h, st, self.p_lin, self.p_rgba, self.stream.cuda_stream, self.rank,
                              self.world, self.layout)

    def gather(self):
        """The frame's one collective, then the unpack kernel on rank 0."""
        if self.world == 1:
            return
        s = self.stream.cuda_stream
        g = self.gathered.data_ptr() if self.gathered is not None else 0
        self.comm.gather_tiles_async(self.w, self.h, self.share.data_ptr(), g, s)
        if self.rank == 0:
            self.rtgo.unpack_tiles_async(self.w, self.h, self.world, g, self.img_lin.data_ptr(),
                                         self.img_rgba.data_ptr(), s)

    def counts(self, st):
        return self.ctx.count(self.w, self.h, st, self.p_lin, self.p_rgba, self.stream.cuda_stream, self.rank,
                              self.world, self.layout)


def barrier_sync(torch, dist, world):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(torch, dist, world, x):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # gloo (host): the device data path is RCCL's only
    return float(t.item())


def time_steps(frames, torch, dist, world, sts, warmup):
    """W untimed steps, then K = len(sts) timed steps (step i renders with
    settings sts[i]: its own seed) between barrier + synchronize on both
    sides; step i runs frames[i % F] on its own stream.  Returns
    (max-over-ranks seconds, per-launch kernel ms from HIP events recorded on
    the stream each render runs on)."""
    F = len(frames)
    for i in range(warmup):
        fr = frames[i % F]
        fr.render(sts[i % len(sts)])
        fr.gather()
    barrier_sync(torch, dist, world)
    evs = []
    t0 = time.perf_counter()
    for i, st in enumerate(sts):
        fr = frames[i % F]
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(fr.stream)
        fr.render(st)
        e1.record(fr.stream)
        evs.append((e0, e1))
        fr.gather()
    barrier_sync(torch, dist, world)
    elapsed = max_over_ranks(torch, dist, world, time.perf_counter() - t0)
    return elapsed, [a.elapsed_time(b) for a, b in evs]


def first_frame_ms(rtgo, torch, dist, scene, W, H, st, rank, world, local, comm):
    """One frame on a fresh context: it also builds what the timed steps
    reuse (frustum masks, the one-sample pilot render, block building and
    upload).  Wall clock, max over ranks."""
    ctx = rtgo.Context(local)
    ctx.set_scene(scene)
    frame = Frame(rtgo, torch, ctx, W, H, rank, world, local, torch.cuda.Stream(), comm)
    barrier_sync(torch, dist, world)
    t0 = time.perf_counter()
    frame.render(st)
    frame.gather()
    torch.cuda.synchronize()
    ms = max_over_ranks(torch, dist, world, (time.perf_counter() - t0) * 1e3)
    ctx.close()
    return ms


def render_e2e(rtgo, scene, W, H, args, local):
    """The blocking Render of the C ABI (N = 1): scene check + upload,
    schedule, kernels, image download to the host."""
    st = rtgo.default_settings()
    st.samples, st.max_depth = args.spp, args.depth
    r = rtgo.ParallelRenderer(devices=[local])
    r.settings = st
    t0 = time.perf_counter()
    st.seed = args.seed
    r.render(scene, W, H)  # the first call on a new renderer: context, upload, schedule (pilot)
    first_ms = (time.perf_counter() - t0) * 1e3
    secs, walls = [], []
    for i in range(7):
        r.settings.seed = args.seed + 1 + i
        t0 = time.perf_counter()
        r.render(scene, W, H)
        walls.append(time.perf_counter() - t0)
        secs.append(r.last_stats.render_seconds)
    r.close()
    one = []
    for i in range(5):
        st.seed = args.seed + 100 + i
        _, _, stats = rtgo.render(scene, W, H, st)
        one.append(stats.render_seconds)
    med = statistics.median(secs)
    rays = W * H * args.spp
    return {
        "ms_median": round(med * 1e3, 4),
        "value": round(rays / med / 1e6, 3),
        "unit": "Mrays/s",
        "wall_ms_median": round(statistics.median(walls) * 1e3, 4),
        "first_call_ms": round(first_ms, 3),
        "oneshot_ms_median": round(statistics.median(one) * 1e3, 3),
        "oneshot_value": round(rays / statistics.median(one) / 1e6, 3),
        "note": "rt_renderer_render (NewParallelRenderer once, Render per frame): rt_stats.render_seconds, "
                "median of 7 calls with distinct seeds; includes the scene check and the device->host copy "
                "of the float3 + RGBA8 image (pageable host memory). first_call_ms: the first Render of a new "
                "renderer (device context, scene upload, schedule + pilot). oneshot: rt_render, which "
                "creates and destroys the device context every call (median of 5).",
    }


def flops_of(counts):
    return sum(FLOPS_PER_EVENT[k] * counts.get(k, 0) for k in FLOPS_PER_EVENT)


def host_threads(args):
    """CPU threads for the baseline: the box's share of host cores."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = args.cpu_threads or (min(share, aff) if share > 0 else aff)
    return threads, aff


def cpu_baseline(args, rtgo, scene, W, H, st, cfg):
    """The oracle (C restatement of the Go goroutine path, linear hitWorld
    scan) on the host cores, on a bounded sample of the same workload."""
    import oracle

    threads, aff = host_threads(args)
    n_tiles = rtgo.num_tiles(W, H)
    if cfg in ("c4", "c5"):
        # 10k-sphere linear scan: ~3 CPU-s per tile-sample-pass; time 2
        # tiles per thread at 4 spp (every (n/(2T))-th tile, full depth),
        # scaled per primary sample
        spp = 4
        stb = rtgo.default_settings()
        stb.samples, stb.max_depth, stb.seed = spp, st.max_depth, st.seed
        ntl = 2 * threads
        world = max(1, n_tiles // ntl)
        t0 = time.perf_counter()
        oracle.render(scene, W, H, stb, rank=0, world=world, nthreads=threads, max_tiles=ntl)
        secs = time.perf_counter() - t0
        rays = ntl * 1024 * spp
        sample = (f"{ntl} tiles (every {world}th tile from tile 0) of the {W}x{H} frame at {spp} spp, depth "
                  f"{st.max_depth}, one run ({secs:.1f} s), scaled per primary sample")
    else:
        oracle.render(scene, W, H, st, nthreads=threads, max_tiles=16)  # warm-up
        times = []
        for _ in range(3):
            t0 = time.perf_counter()
            oracle.render(scene, W, H, st, nthreads=threads)
            times.append(time.perf_counter() - t0)
        secs = sorted(times)[1]
        rays = W * H * st.samples
        sample = f"full {W}x{H}x{st.samples}spp frame, median of 3 runs ({secs:.2f} s) after 1 warm-up"
    return {
        "value": round(rays / secs / 1e6, 3),
        "unit": "Mrays/s",
        "cores": threads,
        "host_cpus": {"affinity": aff, "os_cpu_count": os.cpu_count()},
        "kind": "port",
        "sample": sample + f"; oracle/oracle.c on {threads} threads (tile queue of renderer.go:67-148; the Go "
                           f"toolchain is absent, SURVEY.md §8c)",
    }


def cpu_baseline_bvh(args, rtgo, scene, W, H, st):
    """Secondary CPU baseline of the 10k-sphere configs: the
    oracle with a sphere BVH and any-hit shadow rays (oracle_render_ex, the
    same image), on the same tile sample as cpu_baseline but at the config's
    full spp, so the GPU speedup's algorithmic share is visible."""
    import oracle

    threads, aff = host_threads(args)
    ntl = 2 * threads
    world = max(1, rtgo.num_tiles(W, H) // ntl)
    t0 = time.perf_counter()
    oracle.render(scene, W, H, st, rank=0, world=world, nthreads=threads, max_tiles=ntl, bvh=True)
    secs = time.perf_counter() - t0
    rays = ntl * 1024 * st.samples
    return {
        "value": round(rays / secs / 1e6, 3),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port+bvh",
        "sample": f"{ntl} tiles (every {world}th tile from tile 0) of the {W}x{H} frame at {st.samples} spp, depth "
                  f"{st.max_depth}, one run ({secs:.1f} s); oracle/oracle.c with a median-split sphere BVH and "
                  f"any-hit shadow rays on {threads} threads (not the reference's linear scans; same image)",
    }


def pmc_traffic(workload):
    """HBM bytes per launch from the committed rocprofv3 PMC passes
    (profiles/r02_pmc_traffic.json, scripts/pmc_traffic.py, with the gfx950
    corrections of MI355X_MICROARCH.md §HBM), if they match this workload."""
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
        # host-side coordination only (barriers, the max over ranks, the RCCL
        # id); the frame's data moves through librtgo's RCCL communicator
        dist.init_process_group("gloo")

    cfg = args.config
    spec, W, H, spp, label, steps_default, fif_default = CONFIGS[cfg]
    args.spp = args.spp or spp
    steps = args.steps or steps_default
    if args.warmup < 0:
        args.warmup = 1 if cfg in ("c4", "c5") else 3
    strong = args.strong or cfg in ("c4", "c5")
    if not strong:
        H = H * world  # weak scaling: N-fold vertical sample density
    sts = []
    for i in range(steps):
        st = rtgo.default_settings()
        st.samples, st.max_depth, st.seed = args.spp, args.depth, args.seed + i
        st.num_workers = world
        sts.append(st)
    F = max(1, args.frames_in_flight or fif_default)
    scene = load_scene(rtgo, spec)

    comms = [None] * F
    if world > 1:
        for j in range(F):  # one communicator per frame slot (frames in flight never share one)
            uid = [rtgo.Comm.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            comms[j] = rtgo.Comm(uid[0], world, rank, local)

    frames = []
    for j in range(F):  # F frames in flight: own context (schedule), stream and buffers each
        ctx = rtgo.Context(local)
        ctx.set_scene(scene)
        fr = Frame(rtgo, torch, ctx, W, H, rank, world, local, torch.cuda.Stream(), comms[j])
        fr.render(sts[0])  # set-up: builds this context's schedule (like the scene upload)
        fr.gather()
        frames.append(fr)
    counts = frames[0].counts(sts[0])  # algorithmic work of this rank's launch (counting variant, untimed)
    barrier_sync(torch, dist, world)
    elapsed, kms = time_steps(frames, torch, dist, world, sts, args.warmup)
    # the same frames one at a time (the reference's synchronous Render)
    elapsed1, kms1 = time_steps(frames[:1], torch, dist, world, sts, args.warmup) if F > 1 else (elapsed, kms)
    first_ms = first_frame_ms(rtgo, torch, dist, scene, W, H, sts[0], rank, world, local, comms[0])
    e2e = None
    if world == 1 and not args.no_e2e and cfg in ("c2", "c2_committed", "c3"):
        e2e = render_e2e(rtgo, scene, W, H, args, local)

    rays = W * H * args.spp  # all ranks together
    value = rays * steps / elapsed / 1e6
    kernel1_s = sum(kms1) / len(kms1) / 1e3  # this rank's average launch, one frame at a time
    kernelF_s = sum(kms) / len(kms) / 1e3     # ... with F frames in flight
    flops = flops_of(counts)
    achieved_tf = flops / kernel1_s / 1e12
    npix_local = rtgo.tiles_for_rank(W, H, rank, world) * 1024 if world > 1 else W * H
    # algorithmic HBM bytes: framebuffer write (float3 + RGBA8 = 16 B/pixel)
    # + the flattened scene read once per workgroup-resident copy (<= 4 KB)
    hbm_bytes = npix_local * 16 + 4096
    achieved_gbs = hbm_bytes / kernel1_s / 1e9
    workload = "%s %dx%d %dspp depth %d" % (label, W, H, args.spp, args.depth)

    cpu = cpu_bvh = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, rtgo, scene, W, H, sts[0], cfg)
        cpu_bvh = cpu_baseline_bvh(args, rtgo, scene, W, H, sts[0]) if cfg in ("c4", "c5") else None

    if rank == 0:
        out = {
            "metric": "Mrays/sec at 800x600x100spp max_depth=50 (sphere_reflections_light)" if cfg == "c2"
            else "Mrays/sec (%s)" % cfg,
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / steps * 1e3, 4),
            "first_frame_ms": round(first_ms, 4),
            "frames_in_flight": F,
            "one_frame_in_flight": {
                "value": round(rays * steps / elapsed1 / 1e6, 3),
                "ms_per_step": round(elapsed1 / steps * 1e3, 4),
                "kernel_ms": round(kernel1_s * 1e3, 4),
            },
            "render_e2e": e2e,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,  # BASELINE.md has no published number on this hardware/config
            "dtype": "f64",
            "data": "synthetic: the reference's scene JSON%s, seeded counter-keyed RNG (seed %d + step: every "
                    "step a different image)" % (" (camera facing the objects)" if "facing" in spec else "",
                                                 args.seed),
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
                "kernel": KERNELS[cfg],
                "kernel_ms": round(kernel1_s * 1e3, 4),
                "kernel_ms_frames_in_flight": round(kernelF_s * 1e3, 4),
                "flops_per_launch": flops,
                "note": "FP64 VALU-bound branchy path (binary64 like the Go reference; no matrix shape, no MFMA). "
                        "achieved = algorithmic FP64 ops of one launch (the kernel's own event counts x DESIGN.md "
                        "§4.5 per-event costs, executed work only: culled tests are not counted) / average launch "
                        "time one frame at a time (HIP events on the render stream). kernel_ms_frames_in_flight: "
                        "the same launches overlapped (they share the GPU with their neighbours' tails). "
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
            "cpu_baseline": cpu,
        }
        if cpu:
            out["gpu_over_cpu"] = round(value / cpu["value"], 1)
            if e2e:
                out["render_e2e"]["vs_cpu"] = round(e2e["value"] / cpu["value"], 1)
        if cpu_bvh:
            out["cpu_baseline_bvh"] = cpu_bvh
            out["gpu_over_cpu_bvh"] = round(value / cpu_bvh["value"], 1)
        print(json.dumps(out), flush=True)
    for c in comms:
        if c is not None:
            c.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
