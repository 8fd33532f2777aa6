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
          B consecutive steps (frames that differ only in their seed) form one
          launch (rt_context_render_frames_async; --frames-per-launch, default
          16 for c2/c3), and F launches are in
          flight (--frames-in-flight; default 2 at one GPU, 3 at N > 1): launch
          j runs on slot j % F (own context, stream and buffers), so a frame's
          low-occupancy tail (its last 50-bounce paths) is
          paid once per launch and overlaps the next launch's start.  The same
          frames are also timed one at a time (the reference's synchronous
          Render): "one_frame_in_flight".
          For N > 1 a launch also includes its one RCCL gather of the ranks'
          packed shares to rank 0 (librtgo's ncclSend/ncclRecv group over
          xGMI, on one gather stream per rank, in step order) and the unpack
          kernel there.  The work schedule of a (scene, frame,
          settings) key is built by the first frame and reused (seeds
          excluded from the key).
scaling : STRONG by default: every N renders the config's frame (800x600x100
          for c2, BASELINE configs[1]), its 32x32 tiles partitioned over the
          ranks.  Linear-scan scenes use a work-balanced partition
          (rt_partition_balanced: a whole-frame pilot, tiles dealt heaviest
          first to the least loaded rank; every rank plans the same one, which
          is checked); BVH scenes (c4, c5: thousands of busy tiles) the
          strided deal t % N.  --weak renders 800 x (600 N)
          instead (per-GPU work fixed).  value = the frame's samples x steps /
          max-over-ranks time.
end to end: "render_e2e" (N=1): the blocking Render of the C ABI
          (rt_renderer_render: scene check + upload, schedule, kernels,
          device->host copy of the image), median of 7 calls with distinct
          seeds on one renderer object (NewParallelRenderer once, Render per
          frame, as cmd/raytracer uses it); "oneshot" = rt_render, which also
          creates and destroys the device contexts every call.
cpu     : the oracle (oracle/oracle.c: the reference's goroutine tile loop
          restated in C) on runtime.NumCPU() threads = the affinity count of
          this process (cmd/raytracer/main.go:46, BASELINE configs[0]
          "workers=host cores"), rank 0 at N=1 only.

usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c2_committed|c3|c4|c5] [--weak]
Multi-GPU: python bench.py --gpus N starts the N rank processes itself
          (launch_ranks: one child per GPU, started before any GPU call, rank
          0's JSON line forwarded, non-zero exit if any rank fails), or
          python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import hashlib
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

# Operations per counted event: the adds, muls, divides
# and square roots of the reference's formulas, 1 each, for the work the
# kernel EXECUTES (rt_counts minus rt_counts.culled: primitives and camera
# samples culled as provably missed are neither executed nor counted).
FLOPS_PER_EVENT = {
    "camera_rays": 12,     # u, v (2 add + 2 div) + getRay (8)
    "sphere_tests": 20,    # Sphere.Hit up to the discriminant test (+ avg root work)
    "triangle_tests": 46,  # Moller-Trumbore to the t test
    "shade_events": 75,    # hit record + scatter + path update
    "light_evals": 60,     # direct-lighting terms per light
    "shadow_rays": 15,     # soft direction: scale, add, normalize
    "rng_draws": 5,        # unit conversion + rejection arithmetic
}
# BVH node slab tests run in binary32 on quantized bounds:
# priced against the FP32 peak, in a term of their own
FLOPS_PER_BOX = 12          # 6 fma + 6 min/max/compare
# a ray the soft-shadow traversal kernel sets up: light vector (12), the
# jittered direction (15), inverse direction (3), the binary64 root box (12)
SOFT_RAY_SETUP_FLOPS = 42
# a ray the closest-hit / hard-ray traversal sets up: |d|^2 and its
# reciprocal (6), the inverse direction (3), the binary64 root box (12)
TRAV_RAY_SETUP_FLOPS = 21
PEAK_FP64_TFLOPS = 78.6   # MI355X FP64 vector (= FP64 matrix) peak: 256 CU x 2.4 GHz x 128 FLOP/clk
PEAK_FP32_TFLOPS = 157.3  # MI355X FP32 vector peak (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
PMC_FILE = os.path.join(ROOT, "profiles", "r06_pmc_traffic.json")
# the driver's own command under rocprofv3 --kernel-trace: its timed launches
# (scripts/batched_trace.py, scripts/profile.sh "driver")
TRACE_FILE = os.path.join(ROOT, "profiles", "r06_driver_batched_trace.json")

CONFIGS = {
    # name: (scene, W, H, spp, label, default steps, default frames in flight at one GPU)
    "c2": ("sphere_reflections_light_facing.json", 800, 600, 100, "sphere_reflections_light_facing", 100, 2),
    "c2_committed": ("sphere_reflections_light.json", 800, 600, 100,
                     "sphere_reflections_light as committed (black: objects behind the -Z camera)", 100, 2),
    "c3": ("final_silver_prism_purple_cube_facing.json", 1200, 900, 100, "final_silver_prism_purple_cube_facing",
           50, 2),
    "c4": ("gen:10000", 1920, 1080, 64, "procedural 10k spheres (scenes/gen_spheres.py, BVH)", 3, 1),
    "c5": ("gen:10000", 3840, 2160, 256, "procedural 10k spheres (scenes/gen_spheres.py, BVH)", 1, 1),
}
WAVEFRONT = ("c4", "c5")
KERNELS = {  # the dominant kernel of each config (rocprofv3 --stats, profiles/)
    "c2": "rtgo::render_kernel<false, true, false, false>",
    "c2_committed": "rtgo::render_kernel<false, true, false, false>",
    "c3": "rtgo::render_kernel<false, true, false, false>",
    # the soft-shadow stage: cone walks, list tests, traced soft rays
    "c4": "rtgo::wf_cone4<false> + rtgo::wf_listtest<false> + rtgo::wf_widetest<false> + "
          "rtgo::wf_occlude4<false, true>",
    "c5": "rtgo::wf_cone4<false> + rtgo::wf_listtest<false> + rtgo::wf_widetest<false> + "
          "rtgo::wf_occlude4<false, true>",
}
SOFT_STAGE = ("cone", "cone_rays", "occlude_soft")  # its kernel classes (rtgo.WF_KERNELS)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=0, help="timed steps (default per config: c2 100)")
    ap.add_argument("--warmup", type=int, default=-1, help="untimed steps (default: c2/c3 3, c4/c5 1)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--spp", type=int, default=0, help="override the config's spp")
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--weak", action="store_true", help="c2/c3: frame W x (H*N) (per-GPU work fixed)")
    ap.add_argument("--strided", action="store_true", help="N > 1: deal tiles t %% N instead of by estimated work")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (default: the affinity count)")
    ap.add_argument("--frames-in-flight", type=int, default=0,
                    help="launches in flight per rank (own context, stream and buffers each)")
    ap.add_argument("--frames-per-launch", type=int, default=0,
                    help="frames of one launch (rt_context_render_frames_async, at most 16)")
    ap.add_argument("--host-gather", action="store_true",
                    help="TEST MODE (not a bench line): gather the shares over gloo host copies instead of RCCL, "
                         "so N ranks can share one GPU (RCCL refuses two ranks on one device); --check compares "
                         "rank 0's last image with a 1-rank render")
    ap.add_argument("--check", action="store_true", help="(default at N > 1; kept for old command lines)")
    ap.add_argument("--tuning", default="",
                    help="rt_tuning overrides KEY=VAL[,KEY=VAL] for every context (work partition only: never "
                         "changes an image; sweeps)")
    ap.add_argument("--watchdog", type=float, default=120.0,
                    help="N > 1: a rank's blocking wait (a launch, a gather, a barrier) that has not completed in "
                         "this many seconds prints the rank, step and partition and exits with status 3 "
                         "(rtgo/watchdog.py; <= 0: unbounded)")
    ap.add_argument("--withhold-rank", type=int, default=-1,
                    help="TEST MODE with --host-gather: this rank never joins the gathers (the watchdog must fire)")
    ap.add_argument("--no-check", action="store_true",
                    help="N > 1: skip the post-run check of the last frame against a 1-rank render")
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="TEST MODE of the rank launcher: every rank prints its launch environment as one JSON line "
                         "and exits before anything touches a GPU")
    ap.add_argument("--dry-run-fail-rank", type=int, default=-1,
                    help="TEST MODE with --launch-dry-run: this rank exits with status 5")
    ap.add_argument("--dry-run-hang-rank", type=int, default=-1,
                    help="TEST MODE with --launch-dry-run: this rank sleeps (the launcher must end it)")
    return ap.parse_args()


# ------------------------------------------------------------ rank launcher
# `python bench.py --gpus N` (N > 1) without torch.distributed.run: this
# process starts the N ranks itself, one child process per GPU, BEFORE it
# touches torch.cuda / HIP / RCCL (it never imports torch).  Each child gets
# the environment torch.distributed.run would give it; the parent forwards
# rank 0's stdout (the one JSON line) as its only stdout, the other ranks'
# output to stderr, and exits non-zero if any rank fails (the first failing
# rank's status; a rank whose watchdog fired exits 3).  The torch.distributed
# .run route (WORLD_SIZE set) is untouched.
LAUNCH_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "MASTER_ADDR", "MASTER_PORT",
              "GPU_MAX_HW_QUEUES", "HSA_ENABLE_IPC_MODE_LEGACY", "TORCHELASTIC_RUN_ID")


def free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(n, port, base=None):
    """The environment of each of the n ranks (what torch.distributed.run
    --nnodes 1 --nproc-per-node n --master-addr 127.0.0.1 sets)."""
    base = dict(os.environ if base is None else base)
    out = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TORCHELASTIC_RUN_ID="bench-launcher")
        # several launches and a gather stream in flight per rank;
        # set before HIP starts in the child (at most 32 on this pool)
        e.setdefault("GPU_MAX_HW_QUEUES", "16")
        # the host driver supports dmabuf IPC only (RCCL between processes)
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        e["PYTHONUNBUFFERED"] = "1"
        out.append(e)
    return out


def launch_ranks(args, argv, grace_s=30.0):
    """Start args.gpus rank processes of this script, forward rank 0's stdout,
    return the job's exit status (0 only if every rank exited 0).  When a rank
    fails, the others get `grace_s` seconds to end on their own (their
    watchdogs), then are terminated by PID.  If the launcher is itself
    stopped (SIGTERM / SIGINT / SIGHUP) it ends its ranks first, and a rank
    whose launcher dies anyway gets SIGTERM from the kernel (PDEATHSIG)."""
    import signal
    import subprocess
    import threading

    n = args.gpus
    port = int(os.environ.get("MASTER_PORT", "0")) or free_port()
    procs = []

    def die_with_parent():  # (in the child, before exec: PR_SET_PDEATHSIG = 1)
        import ctypes

        ctypes.CDLL(None).prctl(1, signal.SIGTERM)

    def stop_all(signum, _frame):
        # the launcher itself is being stopped (a driver's time limit): its
        # ranks live in sessions of their own, so end them here, by PID
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except OSError:
                    pass
        t_end = time.monotonic() + 10
        while time.monotonic() < t_end and any(p.poll() is None for p in procs):
            time.sleep(0.1)
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except OSError:
                    pass
        os._exit(128 + signum)

    for sig in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(sig, stop_all)
    for r, env in enumerate(rank_envs(n, port)):
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(),
                                      stderr=None, start_new_session=True, preexec_fn=die_with_parent))

    def pump(p):
        for line in iter(p.stdout.readline, b""):
            sys.stdout.buffer.write(line)
            sys.stdout.flush()

    t = threading.Thread(target=pump, args=(procs[0],), daemon=True)
    t.start()
    status, first_fail, t_fail = [None] * n, None, None
    while any(s is None for s in status):
        for r, p in enumerate(procs):
            if status[r] is None and p.poll() is not None:
                status[r] = p.returncode
                if p.returncode != 0 and first_fail is None:
                    first_fail, t_fail = r, time.monotonic()
                    print(f"[launcher] rank {r} exited with status {p.returncode}", file=sys.stderr, flush=True)
        if first_fail is not None and time.monotonic() - t_fail > grace_s:
            for r, p in enumerate(procs):
                if status[r] is None:
                    print(f"[launcher] terminating rank {r} (pid {p.pid})", file=sys.stderr, flush=True)
                    try:
                        os.killpg(p.pid, signal.SIGTERM)
                    except OSError:
                        pass
            first_fail_grace = time.monotonic()
            while any(s is None for s in status) and time.monotonic() - first_fail_grace < 10:
                for r, p in enumerate(procs):
                    if status[r] is None and p.poll() is not None:
                        status[r] = p.returncode
                time.sleep(0.1)
            for r, p in enumerate(procs):
                if status[r] is None:
                    try:
                        os.killpg(p.pid, signal.SIGKILL)
                    except OSError:
                        pass
                    status[r] = p.wait()
            break
        time.sleep(0.05)
    t.join(timeout=10)
    if first_fail is not None:
        code = status[first_fail]
        return code if isinstance(code, int) and code > 0 else 1
    return 0


def dry_run_rank(args):
    """--launch-dry-run in a rank: report the launch environment, no GPU."""
    rank = int(os.environ.get("RANK", "0"))
    line = {"rank": rank, "pid": os.getpid(), "env": {k: os.environ.get(k) for k in LAUNCH_ENV}}
    print(json.dumps(line), flush=True)
    if rank == args.dry_run_hang_rank:
        time.sleep(600)
    return 5 if rank == args.dry_run_fail_rank else 0


def load_scene(rtgo, spec):
    if spec.startswith("gen:"):
        from scene_cases import spheres10k_scene

        return spheres10k_scene(rtgo, int(spec[4:]))
    return rtgo.Scene.load_from_file(os.path.join(ROOT, "scenes", spec))


class Slot:
    """One launch slot of this rank: its context (schedule), render stream and
    buffers for up to B frames per launch (rt_context_render_frames_async).
    world 1: B W*H images.  world > 1: this rank's packed shares of the
    partition, its B frames contiguous ([B][share]); rank 0 renders them in
    place into its gather buffer [world][B][share] and unpacks the B images
    there in one launch."""

    def __init__(self, rtgo, torch, scene, w, h, rank, world, device, part, B):
        self.rtgo, self.w, self.h, self.rank, self.world, self.part, self.B = rtgo, w, h, rank, world, part, B
        self.ctx = rtgo.Context(device)
        if TUNING:
            self.ctx.set_tuning(rtgo.default_tuning(**TUNING))
        self.ctx.set_scene(scene)
        self.stream = torch.cuda.Stream(device)
        self.rendered = torch.cuda.Event()
        self.gathered = None  # event: the shares have been sent (and unpacked on rank 0)
        self.n = 0            # frames of the last launch
        dev = torch.device("cuda", device)
        if world == 1:
            self.layout = rtgo.RT_LAYOUT_IMAGE
            self.lin = torch.zeros((B, w * h * 3), dtype=torch.float32, device=dev)
            self.rgba = torch.zeros((B, w * h * 4), dtype=torch.uint8, device=dev)
            self.p_lin = [self.lin[f].data_ptr() for f in range(B)]
            self.p_rgba = [self.rgba[f].data_ptr() for f in range(B)]
            return
        self.ctx.set_partition(part)
        self.layout = rtgo.RT_LAYOUT_PACKED_TILES
        nb = part.packed_bytes
        self.share_bytes = nb
        if rank == 0:
            self.gbuf = torch.zeros(world * B * nb, dtype=torch.uint8, device=dev)
            self.share = self.gbuf[:B * nb]
            self.img_lin = torch.zeros((B, w * h * 3), dtype=torch.float32, device=dev)
            self.img_rgba = torch.zeros((B, w * h * 4), dtype=torch.uint8, device=dev)
        else:
            self.gbuf = None
            self.share = torch.zeros(B * nb, dtype=torch.uint8, device=dev)
        base = self.share.data_ptr()
        self.p_lin = [base + f * nb for f in range(B)]
        self.p_rgba = [p + part.rgba_offset for p in self.p_lin]

    def render(self, sts):
        """One launch of the frames sts (<= B; they differ only in seed)."""
        if self.gathered is not None:  # the buffers are free again once their last gather is done
            self.stream.wait_event(self.gathered)
        n = self.n = len(sts)
        self.ctx.render_frames_async(self.w, self.h, sts[0], [st.seed for st in sts], self.p_lin[:n],
                                     self.p_rgba[:n], self.stream.cuda_stream, self.rank, self.world, self.layout)

    def gather(self, torch, comm, gstream):
        """The launch's one collective (on the rank's gather stream, in step
        order: each rank sends its n frames' shares, contiguous), then one
        unpack kernel for the n images on rank 0."""
        if self.world == 1:
            return
        self.rendered.record(self.stream)
        gstream.wait_event(self.rendered)
        g = self.gbuf.data_ptr() if self.gbuf is not None else 0
        nbytes = self.n * self.share_bytes
        if isinstance(comm, HostGather):
            comm.gather(torch, self, gstream, nbytes)
        else:
            comm.gather_bytes_async(nbytes, self.share.data_ptr(), g, gstream.cuda_stream)
        if self.rank == 0:
            self.part.unpack_frames_async(self.n, g, self.img_lin.data_ptr(), self.img_rgba.data_ptr(),
                                          gstream.cuda_stream)
        if self.gathered is None:
            self.gathered = torch.cuda.Event()
        self.gathered.record(gstream)

    def image(self, f):
        """(linear, rgba) device tensors of frame f of the last launch (rank 0)."""
        if self.world == 1:
            return self.lin[f], self.rgba[f]
        return self.img_lin[f], self.img_rgba[f]

    def counts(self, st):
        return self.ctx.count(self.w, self.h, st, self.p_lin[0], self.p_rgba[0], self.stream.cuda_stream, self.rank,
                              self.world, self.layout, full=True)

    def close(self):
        self.ctx.close()


class HostGather:
    """--host-gather (test mode): the same gather through torch.distributed
    gloo and host copies, synchronous; lets N ranks share one GPU."""

    def __init__(self, dist, rank, world):
        self.dist, self.rank, self.world = dist, rank, world

    def gather(self, torch, slot, gstream, nbytes):
        from rtgo.watchdog import host_gather

        with torch.cuda.stream(gstream):
            host = slot.share[:nbytes].cpu()
        if self.rank == WITHHOLD:  # test mode: this rank never sends (the others' watchdogs must fire)
            return
        parts = host_gather(self.dist, host, self.rank, self.world)
        if self.rank == 0:
            with torch.cuda.stream(gstream):
                for r in range(1, self.world):
                    slot.gbuf[r * nbytes:(r + 1) * nbytes].copy_(parts[r].to(slot.gbuf.device))

    def close(self):
        pass


def barrier_sync(torch, dist, world, phase="barrier", **info):
    with WD.guard(phase, **info):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()


def max_over_ranks(torch, dist, world, x):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64)
    with WD.guard("max over ranks", step="report", partition=PART_INFO):
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # gloo (host): the device data path is RCCL's only
    return float(t.item())


def launches(sts, B):
    """The K steps as ceil(K / B) launches of consecutive frames, of near-equal
    size (20 steps at B = 16: 10 + 10, not 16 + 4), so a launch's tail is
    spread evenly and the line does not depend on K mod B."""
    n = len(sts)
    k = -(-n // B) if n else 0
    out, i = [], 0
    for j in range(k):
        m = -(-(n - i) // (k - j))
        out.append(sts[i:i + m])
        i += m
    return out


def busy_ms(spans):
    """Union length (ms) of [start, end) intervals: the time at least one
    launch of the timed region was running (launches in flight overlap)."""
    tot, cur_s, cur_e = 0.0, None, None
    for a, b in sorted(spans):
        if cur_e is None or a > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def time_steps(slots, torch, dist, world, sts, warmup, comm, gstream, B):
    """W untimed steps, then K = len(sts) timed steps (step i renders with
    settings sts[i]: its own seed) between barrier + synchronize on both
    sides; B consecutive steps form one launch, launch j runs on
    slots[j % F].  Returns (max-over-ranks seconds, per-frame kernel ms of
    each launch from HIP events recorded on the stream it runs on)."""
    F = len(slots)
    for j, batch in enumerate(launches([sts[i % len(sts)] for i in range(warmup)], B)):
        sl = slots[j % F]
        with WD.guard("warm-up launch", step=f"warm-up launch {j}", partition=PART_INFO):
            sl.render(batch)
            sl.gather(torch, comm, gstream)
    barrier_sync(torch, dist, world, "warm-up barrier", step="after warm-up", partition=PART_INFO)
    evs = []
    ref = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ref.record()
    for j, batch in enumerate(launches(sts, B)):
        sl = slots[j % F]
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        if sl.gathered is not None:
            sl.stream.wait_event(sl.gathered)
        e0.record(sl.stream)
        with WD.guard("timed launch", step=f"launch {j}: steps of seeds {batch[0].seed}..{batch[-1].seed}",
                      partition=PART_INFO):
            sl.render(batch)
            e1.record(sl.stream)
            evs.append((e0, e1, len(batch)))
            sl.gather(torch, comm, gstream)
    barrier_sync(torch, dist, world, "timed-region barrier (every launch and gather enqueued)",
                 step=f"after {len(evs)} timed launches", partition=PART_INFO)
    elapsed = max_over_ranks(torch, dist, world, time.perf_counter() - t0)
    # per-frame kernel time of each launch, and the union of the launches'
    # spans (ms) over the frames: launches in flight overlap, so a launch's
    # own span over its frames over-states the GPU time per frame
    spans = [(ref.elapsed_time(a), ref.elapsed_time(b)) for a, b, _ in evs]
    busy = busy_ms(spans) / max(1, sum(n for _, _, n in evs))
    return elapsed, [a.elapsed_time(b) / n for a, b, n in evs], busy


def first_frame_ms(rtgo, torch, scene, W, H, st, local):
    """One frame on a fresh context (N = 1): it also builds what the timed
    steps reuse (frustum masks, the one-sample pilot render, block building
    and upload).  Wall clock."""
    sl = Slot(rtgo, torch, scene, W, H, 0, 1, local, None, 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sl.render([st])
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    sl.close()
    return ms


def first_frame_ms_multi(rtgo, torch, dist, scene, W, H, st, rank, world, local, comm, gstream, strided):
    """N > 1: one frame on fresh contexts, its partition planned anew (a
    balanced partition measures the frame first, rt_partition_balanced), its
    schedule built, rendered and gathered to rank 0.  Wall clock, max over
    ranks."""
    barrier_sync(torch, dist, world, "first-frame barrier", step="first frame", partition=PART_INFO)
    t0 = time.perf_counter()
    with WD.guard("first frame", step="first frame (fresh contexts)", partition=PART_INFO):
        part, _ = plan_partition(rtgo, torch, dist, scene, W, H, st, rank, world, local, strided)
        sl = Slot(rtgo, torch, scene, W, H, rank, world, local, part, 1)
        sl.render([st])
        sl.gather(torch, comm, gstream)
        torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    sl.close()
    return max_over_ranks(torch, dist, world, ms)


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
    secs, walls, secs_lin = [], [], []
    for i in range(7):
        # Go's Render returns the RGBA image only (renderer.go:67): so does this
        # timed call; the same call with the float3 image too is timed beside it
        r.settings.seed = args.seed + 1 + i
        t0 = time.perf_counter()
        r.render(scene, W, H, keep_linear=False)
        walls.append(time.perf_counter() - t0)
        secs.append(r.last_stats.render_seconds)
        r.render(scene, W, H)
        secs_lin.append(r.last_stats.render_seconds)
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
        "ms_median_with_linear": round(statistics.median(secs_lin) * 1e3, 4),
        "first_call_ms": round(first_ms, 3),
        "oneshot_ms_median": round(statistics.median(one) * 1e3, 3),
        "oneshot_value": round(rays / statistics.median(one) / 1e6, 3),
        "note": "rt_renderer_render (NewParallelRenderer once, Render per frame): rt_stats.render_seconds, "
                "median of 7 calls with distinct seeds; includes the scene check and the device->host copy "
                "of the RGBA8 image into the caller's (pageable) buffer, which is what Go's Render returns "
                "(ms_median_with_linear: the float3 image too). first_call_ms: the first Render of a new renderer, its creation included (device "
                "context, scene upload, schedule + pilot). oneshot: rt_render, which "
                "creates and destroys the device context every call (median of 5).",
    }


def executed(counts):
    """{event: executed count} = the reference's counts minus the culled part."""
    return {k: v - counts.culled_dict()[k] for k, v in counts.as_dict().items()}


def fp_split(ex, soft=None):
    """(binary64 ops, binary32 ops) of executed event counts ex.  soft: the
    soft-shadow stage's own counts (rt_counts.soft_occlusion): shadow_rays =
    the rays it traced through the BVH (their set-up instead of the generic
    per-event cost), sphere_tests = the cone walks' sphere tests + the list
    tests + the traced rays' tests, box_tests = the cone walks' node tests +
    the traced rays' (the cone set-up and the listed rays' directions are
    not counted: an under-count)."""
    if soft is not None:
        jobs = soft["shadow_rays"]
        f64 = jobs * SOFT_RAY_SETUP_FLOPS + soft["sphere_tests"] * FLOPS_PER_EVENT["sphere_tests"]
        f32 = max(0, soft["box_tests"] - jobs) * FLOPS_PER_BOX  # (the root box per ray is binary64: in the set-up)
        return f64, f32
    f64 = sum(FLOPS_PER_EVENT[k] * ex.get(k, 0) for k in FLOPS_PER_EVENT)
    return f64, ex.get("box_tests", 0) * FLOPS_PER_BOX


def cpu_count_info():
    """The CPUs this process may run on (Go's runtime.NumCPU() is the affinity
    count) and the cgroup's CPU quota, if any (cpu.max: quota / period)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return aff, quota


def cpu_time(oracle, scene, W, H, st, threads, runs=3):
    """Median seconds of `runs` oracle renders (after a short warm-up), and
    the last render's (linear, rgba) image."""
    oracle.render(scene, W, H, st, nthreads=threads, max_tiles=min(16, 2 * threads))  # warm-up
    times, img = [], None
    for _ in range(runs):
        t0 = time.perf_counter()
        img = oracle.render(scene, W, H, st, nthreads=threads)[:2]
        times.append(time.perf_counter() - t0)
    return sorted(times)[len(times) // 2], img


def oracle_check(cf, ref, W, H):
    """The GPU frame cf (bench's check frame) against the oracle's render of
    the same settings, bit for bit: float3 linear (the oracle's binary64
    rounded to binary32, as the kernel writes it) and RGBA8, over the pixels
    the oracle rendered (a tile sample leaves the others NaN)."""
    import numpy as np

    ref_lin, ref_rgba = ref
    g = cf["lin"].reshape(H, W, 3)
    m = ~np.isnan(ref_lin).any(axis=2)
    r32 = ref_lin.astype(np.float32)
    same_lin = np.array_equal(g[m].view(np.uint32), r32[m].view(np.uint32))
    same_rgba = np.array_equal(cf["rgba"].reshape(H, W, 4)[m], ref_rgba[m])
    d = g[m].astype(np.float64) - r32[m].astype(np.float64)
    return bool(same_lin and same_rgba), {
        "pixels_compared": int(m.sum()),
        "rmse_max_channel": float(np.sqrt(np.mean(d ** 2, axis=0)).max()) if d.size else 0.0,
        "max_abs_diff": float(np.abs(d).max()) if d.size else 0.0,
    }


def cpu_baseline(args, rtgo, scene, W, H, st, cfg):
    """The oracle (C restatement of the Go goroutine path, linear hitWorld
    scan) on runtime.NumCPU() threads, on a bounded sample of the same workload."""
    import oracle

    aff, quota = cpu_count_info()
    threads = args.cpu_threads or aff
    n_tiles = rtgo.num_tiles(W, H)
    if cfg in WAVEFRONT:
        # 10k-sphere linear scan: ~1.4 CPU-s per tile-sample-pass; time 32
        # tiles at 4 spp (a strided tile sample, full depth: ~180 CPU-s,
        # ~11 s on a 16-CPU share), scaled per primary sample
        spp = 4
        stb = rtgo.default_settings()
        stb.samples, stb.max_depth, stb.seed = spp, st.max_depth, st.seed
        ntl = min(n_tiles, 32)
        world = max(1, n_tiles // ntl)
        t0 = time.perf_counter()
        oracle.render(scene, W, H, stb, rank=0, world=world, nthreads=threads, max_tiles=ntl)
        secs = time.perf_counter() - t0
        rays = ntl * 1024 * spp
        sample = (f"{ntl} tiles (every {world}th tile from tile 0) of the {W}x{H} frame at {spp} spp, depth "
                  f"{st.max_depth}, one run ({secs:.1f} s), scaled per primary sample")
        img = None
        other = None
    else:
        # the frame bench.py checks (its seed), timed on NumCPU() threads and
        # on the box's per-GPU CPU share (16 threads, the cgroup's quota): the
        # faster of the two is the baseline, the other is reported beside it
        secs, img = cpu_time(oracle, scene, W, H, st, threads)
        rays = W * H * st.samples
        sample = f"full {W}x{H}x{st.samples}spp frame (seed {st.seed}), median of 3 runs ({secs:.3f} s) after 1 warm-up"
        other = None
        if threads != 16:
            secs16, _ = cpu_time(oracle, scene, W, H, st, 16)
            other = {"value": round(rays / secs16 / 1e6, 3), "unit": "Mrays/s", "cores": 16,
                     "sample": f"the same frame on 16 threads, median of 3 ({secs16:.3f} s)"}
            if secs16 < secs:
                other, secs, threads = ({"value": round(rays / secs / 1e6, 3), "unit": "Mrays/s", "cores": threads,
                                         "sample": f"the same frame on {threads} threads = runtime.NumCPU(), median "
                                                   f"of 3 ({secs:.3f} s)"}, secs16, 16)
                sample = (f"full {W}x{H}x{st.samples}spp frame (seed {st.seed}), median of 3 runs ({secs:.3f} s) "
                          f"after 1 warm-up")
    out = {
        "value": round(rays / secs / 1e6, 3),
        "unit": "Mrays/s",
        "cores": threads,
        "host_cpus": {"affinity": aff, "os_cpu_count": os.cpu_count(), "cgroup_cpu_quota": quota},
        "kind": "port",
        "sample": sample + f"; oracle/oracle.c on {threads} threads on the tile queue of renderer.go:67-148 "
                           + (f"(the faster of runtime.NumCPU() = {aff} threads, cmd/raytracer/main.go:46, and 16 "
                              f"threads; every ratio in this line divides by this value)" if other else
                              "(runtime.NumCPU(), cmd/raytracer/main.go:46)")
                           + "; the Go toolchain is absent (SURVEY.md §8c)"
                           + (f"; the cgroup grants {quota} CPUs of time" if quota else ""),
    }
    if other:
        out["other_thread_count"] = other
    return out, img


def cpu_secondary(args, rtgo, scene, W, H, st, cfg):
    """Labelled secondary CPU figure: the as-committed C1 scene (BASELINE
    configs[0]) on NumCPU threads."""
    import oracle

    aff, _ = cpu_count_info()
    out = {}
    if cfg == "c2":
        c1 = rtgo.Scene.load_from_file(os.path.join(ROOT, "scenes", "sphere_reflections_light.json"))
        threads = args.cpu_threads or aff
        secs, _ = cpu_time(oracle, c1, W, H, st, threads)
        out["cpu_c1_as_committed"] = {
            "value": round(W * H * st.samples / secs / 1e6, 3), "unit": "Mrays/s", "cores": threads,
            "sample": f"BASELINE configs[0]: sphere_reflections_light.json as committed (every camera ray misses, "
                      f"a black image) {W}x{H}x{st.samples}spp, depth {st.max_depth}, median of 3 ({secs:.3f} s)"}
    return out


def cpu_baseline_bvh(args, rtgo, scene, W, H, st):
    """Secondary CPU baseline of the 10k-sphere configs: the
    oracle with a sphere BVH and any-hit shadow rays (oracle_render_ex, the
    same image), on the same tile sample as cpu_baseline but at the config's
    full spp, so the GPU speedup's algorithmic share is visible."""
    import oracle

    aff, _ = cpu_count_info()
    threads = args.cpu_threads or aff
    n_tiles = rtgo.num_tiles(W, H)
    ntl = min(n_tiles, 32)
    world = max(1, n_tiles // ntl)
    t0 = time.perf_counter()
    img = oracle.render(scene, W, H, st, rank=0, world=world, nthreads=threads, max_tiles=ntl, bvh=True)[:2]
    secs = time.perf_counter() - t0
    rays = ntl * 1024 * st.samples
    return img, {
        "value": round(rays / secs / 1e6, 3),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port+bvh",
        "sample": f"{ntl} tiles (every {world}th tile from tile 0) of the {W}x{H} frame at {st.samples} spp, depth "
                  f"{st.max_depth}, one run ({secs:.1f} s); oracle/oracle.c with a median-split sphere BVH and "
                  f"any-hit shadow rays on {threads} threads (not the reference's linear scans; same image)",
    }


def pmc_traffic(workload):
    """HBM bytes per launch of the dominant kernel from the committed
    rocprofv3 PMC passes (profiles/r06_pmc_traffic.json, scripts/pmc_traffic.py,
    with the gfx950 corrections of MI355X_MICROARCH.md §HBM), if it holds this
    workload."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    e = d.get(workload) if isinstance(d, dict) else None
    return e.get("hbm_bytes_per_launch") if e else None


def pmc_traffic_batched(workload):
    """HBM bytes per FRAME of the dominant kernel in launches of several
    frames (the "| B frames per launch" entry of the same PMC file), and B."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    for k, e in (d.items() if isinstance(d, dict) else ()):
        if k.startswith(workload + " | "):
            return e.get("hbm_bytes_per_frame"), e.get("frames_per_launch")
    return None, None


def trace_batched(cfg):
    """The committed kernel trace of the driver's command (c2): its timed
    launches' per-frame kernel time (union of their spans over the frames)."""
    if cfg != "c2":
        return None
    try:
        with open(TRACE_FILE) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    return {"union_ms_per_frame": d.get("union_ms_per_frame"), "avg_launch_ms_per_frame": d.get("avg_launch_ms_per_frame"),
            "launch_frames": d.get("bench_cmd_line", {}).get("launch_frames"),
            "ms_per_step_of_that_run": d.get("bench_cmd_line", {}).get("ms_per_step"),
            "file": os.path.relpath(TRACE_FILE, ROOT)}


def plan_partition(rtgo, torch, dist, scene, W, H, st, rank, world, local, strided):
    """The frame's tile partition, and the same on every rank: balanced
    (planned by every rank from the same deterministic measuring render,
    rt_partition_balanced; checked by comparing digests) or strided."""
    if strided:
        return rtgo.Partition(W, H, world), "strided t % N"
    ctx = rtgo.Context(local)
    ctx.set_scene(scene)
    part = ctx.balanced_partition(W, H, st, world)
    ctx.close()
    digest = hashlib.sha256(part.owners(W, H).tobytes()).hexdigest()
    allg = [None] * world
    dist.all_gather_object(allg, digest)
    if len(set(allg)) != 1:
        raise SystemExit(f"rank {rank}: balanced partitions differ across ranks: {allg}")
    return part, "balanced (measured work per tile, heaviest tile first to the least loaded rank)"


TUNING = {}  # --tuning overrides (Slot contexts)
WD = None  # the rank's Watchdog (rtgo/watchdog.py; unbounded at N = 1)
PART_INFO = None  # this rank's partition, for the watchdog's report
WITHHOLD = -1  # --withhold-rank (test mode)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # started as `python bench.py --gpus N`: launch the N ranks (no torch,
        # no GPU call in this process)
        sys.exit(launch_ranks(args, sys.argv[1:], float(os.environ.get("BENCH_LAUNCH_GRACE_S", "30"))))
    if args.launch_dry_run:
        sys.exit(dry_run_rank(args))
    for kv in filter(None, args.tuning.split(",")):
        k, _, v = kv.partition("=")
        TUNING[k] = float(v) if "." in v else int(v)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        # a rank keeps several launches and its gather stream in flight: more
        # hardware queues than HIP's default 4 let them run side by side
        # (scripts/rank_share_probe.py); set before HIP starts
        os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
    import torch
    import torch.distributed as dist

    import rtgo

    from rtgo.watchdog import Watchdog

    global WD, PART_INFO, WITHHOLD
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    WD = Watchdog(args.watchdog if world > 1 else 0, rank)
    if args.withhold_rank >= 0 and not args.host_gather:
        raise SystemExit("--withhold-rank is a --host-gather test mode")
    WITHHOLD = args.withhold_rank
    if world != args.gpus:
        print(f"--gpus {args.gpus} needs torch.distributed.run with {args.gpus} processes (WORLD_SIZE={world})",
              file=sys.stderr)
        sys.exit(2)
    if args.host_gather:  # test mode: N ranks may share the box's GPUs
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        # host-side coordination only (barriers, the max over ranks, the RCCL
        # id, the partition check); the frame's data moves through librtgo's
        # RCCL communicator
        # (gloo prints its "[Gloo] Rank r is connected to ..." lines on stdout
        # while the group forms: sent to stderr, so stdout holds the one JSON
        # line only)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
            with WD.guard("process-group start", step="init"):
                dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)

    cfg = args.config
    spec, W, H, spp, label, steps_default, fif_default = CONFIGS[cfg]
    args.spp = args.spp or spp
    steps = args.steps or steps_default
    if args.warmup < 0:
        args.warmup = 1 if cfg in WAVEFRONT else 3
    weak = args.weak and cfg not in WAVEFRONT
    if weak:
        H = H * world  # N-fold vertical sample density
    sts = []
    for i in range(steps):
        st = rtgo.default_settings()
        st.samples, st.max_depth, st.seed = args.spp, args.depth, args.seed + i
        st.num_workers = world
        sts.append(st)
    # F launches in flight of B frames each: a frame's launch ends with the
    # lone chains of its longest paths; B frames in one launch
    # pay that tail once, F launches overlap one launch's tail with the next's
    # start.  A rank's share at N > 1 holds ~1/N of the frame's work but the
    # frame's longest paths, so it needs more frames per launch
    # (scripts/rank_share_probe.py).  BVH frames: one at a time.
    # At one GPU the timed steps fill the F slots: ceil(K / F) frames per
    # launch up to RT_MAX_FRAMES (K = 20: one launch of 20, below; K = 100:
    # four of 25, two at a time -- 25-frame launches measured 2 % faster than
    # 16-frame ones at K = 100).
    if cfg in WAVEFRONT:
        F, B = 1, 1
    elif world > 1:
        F, B = 3, 16
    else:
        # (r05) K steps that fit one launch run as one launch (one tail for
        # all of them): the driver's 20 frames as one launch of 20 measured
        # 228.1 k Mrays/s against 222.5 k as 10 + 10 side by side and 218.8 k
        # as 7 + 7 + 6 (scripts/k20_probe.sh, three runs each); more steps
        # run F = 2 launches in flight, so that each tail overlaps the next
        # launch's start
        F = 1 if steps <= rtgo.RT_MAX_FRAMES else fif_default
        B = -(-steps // (args.frames_in_flight or F))
    F = args.frames_in_flight or F
    B = max(1, min(rtgo.RT_MAX_FRAMES, args.frames_per_launch or B))
    scene = load_scene(rtgo, spec)

    comm = gstream = part = None
    part_kind = None
    if world > 1:
        if args.host_gather:
            comm = HostGather(dist, rank, world)
        else:
            uid = [rtgo.Comm.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            comm = rtgo.Comm(uid[0], world, rank, local)
        gstream = torch.cuda.Stream(local)
        with WD.guard("partition planning", step="set-up"):
            part, part_kind = plan_partition(rtgo, torch, dist, scene, W, H, sts[0], rank, world, local,
                                             args.strided or cfg in WAVEFRONT)
        PART_INFO = f"{part_kind.split(' (')[0]}, {part.local_tiles(rank)} of {rtgo.num_tiles(W, H)} tiles on rank {rank}"

    slots = []
    for i in range(F):  # F launches in flight: own context (schedule), stream and buffers each
        sl = Slot(rtgo, torch, scene, W, H, rank, world, local, part, B)
        with WD.guard("set-up launch", step=f"slot {i} set-up", partition=PART_INFO):
            sl.render(sts[:B])  # set-up: builds this context's schedule (like the scene upload)
            sl.gather(torch, comm, gstream)
        slots.append(sl)
    barrier_sync(torch, dist, world, "set-up barrier", step="set-up", partition=PART_INFO)
    with WD.guard("counting launch", step="counts", partition=PART_INFO):
        counts = slots[0].counts(sts[0])  # algorithmic work of this rank's launch (counting variant, untimed)
    barrier_sync(torch, dist, world, "counting barrier", step="counts", partition=PART_INFO)
    prof_ctx = slots[0].ctx if cfg in WAVEFRONT else None
    if prof_ctx is not None:
        prof_ctx.profile(True)  # per-kernel HIP events in the timed frames (F = 1: every frame on slot 0)
    elapsed, kms, busy_frame_ms = time_steps(slots, torch, dist, world, sts, args.warmup, comm, gstream, B)
    plan = launches(sts, B)
    check_frame = None
    if world == 1:
        # the frame the oracle checks (check_equals_oracle): one from the last
        # launch that ran on the second slot (the first when F = 1), from the
        # middle of that launch, copied now (later timings reuse slot 0)
        want = min(1, len(slots) - 1, len(plan) - 1)
        j = max(i for i in range(len(plan)) if i % len(slots) == want)
        f = len(plan[j]) // 2
        lin_d, rgba_d = slots[j % len(slots)].image(f)
        check_frame = {"seed": plan[j][f].seed, "launch": j, "slot": j % len(slots), "frame_in_launch": f,
                       "frames_in_launch": len(plan[j]), "st": plan[j][f],
                       "lin": lin_d.cpu().numpy(), "rgba": rgba_d.cpu().numpy()}
    kernel_prof = None
    if prof_ctx is not None:
        kernel_prof = prof_ctx.kernel_seconds()
        prof_ctx.profile(False)
    # the same frames one at a time (the reference's synchronous Render)
    elapsed1, kms1, _ = (time_steps(slots[:1], torch, dist, world, sts, args.warmup, comm, gstream, 1)
                         if F * B > 1 else (elapsed, kms, busy_frame_ms))
    if world == 1:
        first_ms = first_frame_ms(rtgo, torch, scene, W, H, sts[0], local)
    else:
        first_ms = first_frame_ms_multi(rtgo, torch, dist, scene, W, H, sts[0], rank, world, local, comm, gstream,
                                        args.strided or cfg in WAVEFRONT)
    check = share_sums = gathered_ok = None
    if world > 1 and not args.no_check:
        # After the timed region, always at N > 1: the last timed frame (slot 0
        # rendered it last, one frame per launch) proves its own image.  Every
        # rank hashes its packed share; rank 0 hashes each rank's slot of the
        # gather buffer the RCCL group filled (the transport check), then
        # compares its unpacked image with a 1-rank render of the same settings
        # on its own device (createRenderTasks' frame, renderer.go:398-436).
        wd_check = WD.guard("post-run check (share hashes, 1-rank render)", step="after the timed region",
                            partition=PART_INFO)
        wd_check.__enter__()
        torch.cuda.synchronize()
        sl = slots[0]
        nb = sl.share_bytes

        def sha(t):
            return hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()[:16]

        share_sums = [None] * world
        dist.all_gather_object(share_sums, sha(sl.share[:nb]))
        if rank == 0:
            got = [sha(sl.gbuf[r * sl.n * nb:r * sl.n * nb + nb]) for r in range(world)]
            gathered_ok = got == share_sums
            lin, rgba = sl.image(0)
            ref = Slot(rtgo, torch, scene, W, H, 0, 1, local, None, 1)
            ref.render([sts[-1]])
            torch.cuda.synchronize()
            check = bool(gathered_ok and torch.equal(lin, ref.lin[0]) and torch.equal(rgba, ref.rgba[0]))
            ref.close()
        ok = [None] * world
        dist.all_gather_object(ok, (check, gathered_ok))
        check, gathered_ok = ok[0]
        wd_check.__exit__(None, None, None)
    e2e = None
    if world == 1 and not args.no_e2e and cfg in ("c2", "c2_committed", "c3"):
        e2e = render_e2e(rtgo, scene, W, H, args, local)

    rays = W * H * args.spp  # the whole frame (all ranks together)
    value = rays * steps / elapsed / 1e6
    kernel1_s = sum(kms1) / len(kms1) / 1e3  # this rank's average launch, one frame at a time
    kernelF_s = sum(kms) / len(kms) / 1e3     # ... with F frames in flight
    rank_kernel_ms = [kernel1_s * 1e3]
    if world > 1:
        allk = [None] * world
        with WD.guard("kernel-time exchange", step="report", partition=PART_INFO):
            dist.all_gather_object(allk, kernel1_s * 1e3)
        rank_kernel_ms = allk
    ex = executed(counts)
    npix_local = (part.local_tiles(rank) * 1024) if world > 1 else W * H
    # algorithmic HBM bytes: framebuffer write (float3 + RGBA8 = 16 B/pixel)
    # + the flattened scene read once per workgroup-resident copy (<= 4 KB)
    hbm_bytes = npix_local * 16 + 4096
    workload = "%s %dx%d %dspp depth %d" % (label, W, H, args.spp, args.depth)
    if cfg in WAVEFRONT:
        # the soft-shadow stage (cone walks, the rays of
        # listed cones against their lists, the other soft rays through the
        # BVH): its own counts over its own launches (HIP events of the timed
        # frames)
        soft = counts.soft_occlusion_dict()
        k_s = sum(kernel_prof[k][0] for k in SOFT_STAGE)
        k_n = kernel_prof["occlude_soft"][1]
        frames_timed = max(1, kernel_prof["resolve"][1])
        per_frame_s = k_s / frames_timed
        f64, f32 = fp_split(ex, soft=soft)
        kern_s, launches_per_frame = per_frame_s, k_n / frames_timed
        flops_unit = "per frame (%.0f launches)" % launches_per_frame
        frame64, frame32 = fp_split(ex)
        # the two largest kernels since r03 on their own counts and HIP-event
        # time (rt_counts.extend / hard_occlusion)
        per_kernel = {}
        for name, cd, rays_key in (("extend", counts.extend_dict(), "bounce_rays"),
                                   ("occlude_hard", counts.hard_occlusion_dict(), "shadow_rays")):
            ks_k = kernel_prof[name][0] / frames_timed
            k64 = cd[rays_key] * TRAV_RAY_SETUP_FLOPS + cd["sphere_tests"] * FLOPS_PER_EVENT["sphere_tests"]
            k32 = max(0, cd["box_tests"] - cd[rays_key]) * FLOPS_PER_BOX  # (the root box: binary64, in the set-up)
            per_kernel[name] = {
                "kernel_ms_per_frame": round(ks_k * 1e3, 3), "rays": cd[rays_key],
                "sphere_tests": cd["sphere_tests"], "box_tests": cd["box_tests"],
                "fp64_flops": k64, "fp32_flops": k32,
                "achieved_tflops": round((k64 + k32) / ks_k / 1e12, 4) if ks_k > 0 else None,
                "frac": round(k64 / ks_k / 1e12 / PEAK_FP64_TFLOPS + k32 / ks_k / 1e12 / PEAK_FP32_TFLOPS, 5)
                if ks_k > 0 else None,
            }
        whole = {"fp64_flops": frame64, "fp32_flops": frame32, "kernels": per_kernel,
                 "frame_kernel_ms": round(kernel1_s * 1e3, 3),
                 "frac_fp64": round(frame64 / kernel1_s / 1e12 / PEAK_FP64_TFLOPS, 5),
                 "frac_fp32": round(frame32 / kernel1_s / 1e12 / PEAK_FP32_TFLOPS, 5),
                 "kernel_ms_per_frame": {k: round(v[0] / frames_timed * 1e3, 3) for k, v in kernel_prof.items()}}
    else:
        f64, f32 = fp_split(ex)
        kern_s = kernel1_s
        flops_unit = "per launch"
        whole = None
    a64, a32 = f64 / kern_s / 1e12, f32 / kern_s / 1e12
    frac64, frac32 = a64 / PEAK_FP64_TFLOPS, a32 / PEAK_FP32_TFLOPS
    achieved_gbs = hbm_bytes / kernel1_s / 1e9

    cpu = cpu_bvh = cpu2 = None
    check_oracle = check_info = None
    if rank == 0 and world == 1:
        # the oracle renders the check frame's settings: the CPU baseline
        # (full frame, c2/c3) or its BVH tile sample (c4/c5) doubles as the check
        ref_img = None
        cst = check_frame["st"]
        if not args.no_cpu_baseline:
            cpu, ref_img = cpu_baseline(args, rtgo, scene, W, H, cst, cfg)
            cpu2 = cpu_secondary(args, rtgo, scene, W, H, sts[0], cfg)
            if cfg in WAVEFRONT:
                ref_img, cpu_bvh = cpu_baseline_bvh(args, rtgo, scene, W, H, cst)
        elif cfg not in WAVEFRONT:
            import oracle

            ref_img = oracle.render(scene, W, H, cst)[:2]
        if ref_img is not None:
            check_oracle, check_info = oracle_check(check_frame, ref_img, W, H)

    if rank == 0:
        parallelism = "1 GPU" if world == 1 else "%d ranks: tiles %s, one %s gather per frame" % (
            world, part_kind, "HOST (gloo, test mode: not a bench line)" if args.host_gather else "RCCL")
        out = {
            "metric": "Mrays/sec at 800x600x100spp max_depth=50 (sphere_reflections_light)" if cfg == "c2"
            else "Mrays/sec (%s)" % cfg,
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / steps * 1e3, 4),
            "first_frame_ms": round(first_ms, 4) if first_ms is not None else None,
            "frames_in_flight": F * B,
            "launches_in_flight": F,
            "frames_per_launch": B,
            "launch_frames": [len(b) for b in plan],
            "one_frame_in_flight": {
                "value": round(rays * steps / elapsed1 / 1e6, 3),
                "ms_per_step": round(elapsed1 / steps * 1e3, 4),
                "kernel_ms": round(kernel1_s * 1e3, 4),
            },
            "render_e2e": e2e,
            "higher_is_better": True,
            "scaling": "weak" if weak else "strong",
            "vs_baseline": None,  # BASELINE.md has no published number on this hardware/config
            "dtype": "f64",
            "data": "synthetic: the reference's scene JSON%s, seeded counter-keyed RNG (seed %d + step: every "
                    "step a different image)" % (" (camera facing the objects)" if "facing" in spec else "",
                                                 args.seed),
            "config": {
                "workload": workload + ", soft shadows, recursive reflections",
                "width": W, "height": H, "spp": args.spp, "max_depth": args.depth,
                "parallelism": parallelism,
                "frames_in_flight": F * B,
                "frames_per_launch": B,
            },
            "roofline": {
                "bound": "valu",
                "achieved": round(a64 + a32, 4),
                "peak": PEAK_FP64_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(frac64 + frac32, 5),
                "frac_fp64": round(frac64, 5),
                "frac_fp32": round(frac32, 5),
                "fp64_flops": f64,
                "fp32_flops": f32,
                "flops_unit": flops_unit,
                "traffic": pmc_traffic(workload),
                # the same kernel in launches of several frames (the timed ones):
                # HBM bytes per frame, and the rocprof trace's per-frame time
                "traffic_batched_per_frame": pmc_traffic_batched(workload)[0],
                "traffic_batched_frames_per_launch": pmc_traffic_batched(workload)[1],
                "trace_batched": trace_batched(cfg) if world == 1 else None,
                "kernel": KERNELS[cfg],
                "kernel_ms": round(kern_s * 1e3, 4),
                "kernel_ms_frames_in_flight": round(kernelF_s * 1e3, 4) if cfg not in WAVEFRONT else None,
                # the timed launches' HIP-event spans, their union over the
                # frames: GPU time per frame with the launches as the bench
                # runs them (overlapping launches counted once)
                "busy_ms_per_frame": round(busy_frame_ms, 4) if cfg not in WAVEFRONT else None,
                "frac_busy": (round(f64 / (busy_frame_ms * 1e-3) / 1e12 / PEAK_FP64_TFLOPS
                                    + f32 / (busy_frame_ms * 1e-3) / 1e12 / PEAK_FP32_TFLOPS, 5)
                              if cfg not in WAVEFRONT and busy_frame_ms > 0 else None),
                # the same frame's executed flops over the bench's own time per frame
                # (value's frames in flight: launches overlap, so no single launch shows it)
                "frac_in_flight": (round(f64 / (elapsed / steps) / 1e12 / PEAK_FP64_TFLOPS
                                         + f32 / (elapsed / steps) / 1e12 / PEAK_FP32_TFLOPS, 5)
                                   if cfg not in WAVEFRONT and world == 1 else None),
                "note": "FP64 VALU-bound branchy path (binary64 like the Go reference; no matrix shape, no MFMA). "
                        "EXECUTED work only: the counting variant's counts minus rt_counts.culled (the camera "
                        "samples of culled pixels it walks only to report the reference's counts), x DESIGN.md "
                        "§4.5 per-event costs; BVH box tests run in binary32 and are priced against the FP32 peak "
                        "(157.3 TF): frac = frac_fp64 + frac_fp32, the share of the kernel's time the VALU would "
                        "need at peak rate.  kernel_ms: the dominant kernel's average launch one frame at a time "
                        "(HIP events on the render stream; for c4/c5 the soft-shadow traversal kernel's time per "
                        "frame from rt_context_profile's events in the timed frames); frac_in_flight: the frame's flops over "
                        "ms_per_step (the throughput line's time per frame).  traffic = HBM bytes per "
                        "launch from rocprofv3 FETCH_SIZE + WRITE_SIZE passes (profiles/r06_pmc_traffic.json; "
                        "traffic_batched_per_frame: the same passes over launches of several frames, per frame).  "
                        "busy_ms_per_frame / frac_busy: the timed launches' HIP-event spans (their union: launches in "
                        "flight overlap) over the frames; trace_batched: the same from the committed rocprofv3 "
                        "kernel trace of this exact command (profiles/r06_driver_batched_trace.json).",
            },
            "roofline_frame": whole,
            "roofline_hbm": {
                "bound": "hbm",
                "achieved": round(achieved_gbs, 3),
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / PEAK_HBM_GBS, 7),
                "algorithmic_bytes_per_launch": hbm_bytes,
            },
            "rank_kernel_ms": [round(x, 4) for x in rank_kernel_ms],
            # N = 1: a frame of the timed region (a batched launch on the second
            # slot) against the oracle's render of its settings, bit for bit
            "check_equals_oracle": check_oracle,
            "check_frame": ({k: v for k, v in check_frame.items() if k not in ("st", "lin", "rgba")}
                            | (check_info or {})
                            | {"oracle": ("full frame (the cpu_baseline leg's last render)" if cfg not in WAVEFRONT
                                          else "the cpu_baseline_bvh leg's tile sample (same image as the linear "
                                               "scan)")}) if check_frame else None,
            "check_equals_one_rank": check,
            "check_gathered_equals_rank_shares": gathered_ok,
            "rank_share_sha256_16": share_sums,
            # (a strided partition carries no estimate: null)
            "rank_estimated_work": ([round(part.work(r)) for r in range(world)]
                                    if world > 1 and part_kind and part_kind.startswith("balanced") else None),
            "counts_rank0": counts.as_dict(),
            "counts_rank0_executed": ex,
            "cpu_baseline": cpu,
        }
        if cpu:
            # (all ratios over cpu_baseline.value: the faster CPU figure)
            out["gpu_over_cpu"] = round(value / cpu["value"], 1)
            out["gpu_over_cpu_one_frame"] = round(out["one_frame_in_flight"]["value"] / cpu["value"], 1)
            out.update(cpu2 or {})
            if e2e:
                out["render_e2e"]["vs_cpu"] = round(e2e["value"] / cpu["value"], 1)
                out["render_e2e"]["oneshot_vs_cpu"] = round(e2e["oneshot_value"] / cpu["value"], 1)
        if cpu_bvh:
            # c4/c5: the honest CPU basis is the oracle WITH a BVH (same image):
            # cpu_baseline leads with it and every gpu_over_cpu ratio divides by
            # it; the reference's own linear scan (a tile sample at 4 spp) is
            # kept beside it, with its ratio, so the BVH's algorithmic share of
            # the speedup stays visible
            out["cpu_baseline_linear_scan"] = cpu
            out["gpu_over_cpu_linear_scan"] = out.pop("gpu_over_cpu")
            out.pop("gpu_over_cpu_one_frame", None)
            cpu_bvh = dict(cpu_bvh, kind="port", algorithm="oracle + median-split sphere BVH, any-hit shadow rays",
                           host_cpus=cpu.get("host_cpus"))
            out["cpu_baseline"] = cpu_bvh
            out["gpu_over_cpu"] = round(value / cpu_bvh["value"], 1)
            out["cpu_basis"] = ("cpu_baseline = the oracle with a sphere BVH on the same tile sample at full spp "
                                "(the same image as the reference's linear scan); gpu_over_cpu divides by it; "
                                "cpu_baseline_linear_scan / gpu_over_cpu_linear_scan: the reference's linear "
                                "hitWorld scan (renderer.go:333-346) on a 4-spp tile sample")
        print(json.dumps(out), flush=True)
    for sl in slots:
        sl.close()
    if comm is not None:
        comm.close()
    if world > 1:
        with WD.guard("final barrier", step="exit", partition=PART_INFO):
            dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
