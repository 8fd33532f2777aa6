#!/usr/bin/env python3
"""Per-workgroup timing of an RT_WG_TIMING build (dev tool).

usage: RTGO_LIB=.../librtgo_timing.so wg_timing.py [scene.json] [W H SPP]
Prints the kernel span, wave duration percentiles, how many waves are in
flight over time (occupancy profile) and the slowest workgroups' tiles.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "concurrent-raytracer-go_amd"))
import torch  # noqa: E402

import rtgo  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "scenes", "sphere_reflections_light_facing.json")
W, H, SPP = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (800, 600, 100)
ctx = rtgo.Context(0)
if os.environ.get("WG_TUNING"):  # e.g. WG_TUNING="split_samples=16,block_work=256"
    ctx.set_tuning(rtgo.default_tuning(**{k: float(v) if "." in v else int(v) for k, v in
                                          (kv.split("=") for kv in os.environ["WG_TUNING"].split(","))}))
if scene == "spheres10k":  # config C4/C5 scene (scenes/gen_spheres.py)
    import importlib.util
    _spec = importlib.util.spec_from_file_location("g", os.path.join(ROOT, "scenes", "gen_spheres.py"))
    _g = importlib.util.module_from_spec(_spec)
    _spec.loader.exec_module(_g)
    ctx.set_scene(rtgo.Scene.from_json_text(_g.dumps(_g.generate(10000))))
else:
    ctx.set_scene(rtgo.Scene.load_from_file(scene))
st = rtgo.default_settings()
st.samples = SPP
lin = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
rgba = torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda")
nwg_max = 200_000
dbg = torch.zeros(nwg_max * 48, dtype=torch.int64, device="cuda")
ctx.set_debug_buffer(dbg.data_ptr())
RANK, WORLD = int(os.environ.get("WG_RANK", "0")), int(os.environ.get("WG_WORLD", "1"))
if os.environ.get("WG_DEPTH"):
    st.max_depth = int(os.environ["WG_DEPTH"])
for _ in range(2):
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    ctx.render_async(W, H, st, lin.data_ptr(), rgba.data_ptr(), 0, RANK, WORLD, rtgo.RT_LAYOUT_PACKED_TILES)
    e1.record()
    torch.cuda.synchronize()
print(f"kernel {e0.elapsed_time(e1):.3f} ms (rank {RANK}/{WORLD}, depth {st.max_depth})")
WPG = int(os.environ.get("WG_WAVES", "1"))  # waves per workgroup of the kernel
d = dbg.cpu().numpy().reshape(-1, WPG, 48)
used = d[:, 0, 0] != 0
d = d[used]
# tail helpers write records of their own ([14] = -1)
helper = d[:, 0, 14] == -1
hd = d[helper]
d = d[~helper]
if len(hd):
    t0h = d[:, :, 0].min()
    hs = (hd[:, 0, 0] - t0h) / 100.0
    he = (hd[:, 0, 2] - t0h) / 100.0
    hf = np.where(hd[:, 0, 1] > 0, (hd[:, 0, 1] - t0h) / 100.0, np.nan)
    print(f"tail helpers: {len(hd)}, start us p0/p50/p100 {hs.min():.1f}/{np.median(hs):.1f}/{hs.max():.1f}, "
          f"end p0/p50/p100 {he.min():.1f}/{np.median(he):.1f}/{he.max():.1f}, first path p0/p50 "
          f"{np.nanmin(hf) if np.isfinite(hf).any() else -1:.1f}/{np.nanmedian(hf) if np.isfinite(hf).any() else -1:.1f}, "
          f"paths {int(hd[:, 0, 7].sum())}, solo us per path {hd[:, 0, 3].sum() / max(1, hd[:, 0, 7].sum()) / 100:.1f}, "
          f"bounces {int(hd[:, 0, 8].sum())}, us per bounce {hd[:, 0, 3].sum() / max(1, hd[:, 0, 8].sum()) / 100:.2f}")
    late = np.argsort(-he)[:8]
    print("  latest helpers (end us, last path start us, depth at export -> end): " + ", ".join(
        f"({he[i]:.0f}, {(hd[i, 0, 4] - t0h) / 100.0:.0f}, {int(hd[i, 0, 5])}->{int(hd[i, 0, 6])})" for i in late))
nwg = d.shape[0]
t0 = d[:, :, 0].min()
start = (d[:, :, 0] - t0) / 100.0  # s_memrealtime: 100 MHz -> microseconds
loop = (d[:, :, 1] - t0) / 100.0
end = (d[:, :, 2] - t0) / 100.0
span = end.max()
dur = (end - start).ravel()
print(f"{scene} {W}x{H}x{SPP}: {nwg} WGs, span {span:.1f} us")
for q in (50, 90, 99, 99.9, 100):
    print(f"  wave duration p{q}: {np.percentile(dur, q):.1f} us")
epi = (end - loop).ravel()
print(f"  epilogue (reduce+write) p50 {np.percentile(epi, 50):.2f} us  p99 {np.percentile(epi, 99):.2f} us")
# waves in flight over time
grid = np.linspace(0, span, 41)
inflight = [int(((start <= t) & (end > t)).sum()) for t in grid]
print("  waves in flight at 2.5% steps:", inflight)
wgdur = end.max(axis=1) - start.min(axis=1)
order = np.argsort(-wgdur)[:10]
print("  slowest WGs (index, us, start us):", [(int(i), round(float(wgdur[i]), 1), round(float(start[i].min()), 1))
                                              for i in order])
hit, light, soft, fill, it = (d[:, :, k].astype(np.float64) for k in (3, 4, 5, 6, 7))
tot = hit.sum() + light.sum() + fill.sum()
print(f"  section clocks: fill {fill.sum() / tot:.1%}  hit {hit.sum() / tot:.1%}  lighting {light.sum() / tot:.1%} "
      f"(soft part {soft.sum() / tot:.1%});  shade iterations {it.sum():.0f}, per iteration hit "
      f"{hit.sum() / max(it.sum(), 1):.0f} light {light.sum() / max(it.sum(), 1):.0f}")
wave_clk = (end - start) * 2100.0  # us -> shader clocks at ~2.1 GHz
print(f"  accounted / wave time: {tot / wave_clk.sum():.1%}")
hard, scat, alive, coop, seq = (d[:, :, k].astype(np.float64) for k in (8, 9, 10, 11, 12))
print(f"  lighting split: cone+hard {hard.sum() / tot:.1%}  soft {soft.sum() / tot:.1%}  rest "
      f"{(light.sum() - hard.sum() - soft.sum()) / tot:.1%};  scatter {scat.sum() / tot:.1%}")
print(f"  lanes alive per shade iteration {alive.sum() / max(it.sum(), 1):.1f}; coop owners {coop.sum():.0f}, "
      f"soft_seq passes {seq.sum():.0f}")
for i in order[:6]:
    for w in range(WPG):
        npx, ns = int(d[i, w, 13]) >> 16, int(d[i, w, 13]) & 0xFFFF
        print(f"    WG {int(i)}: np {npx} ns {ns} split {int(d[i, w, 14]) - 1}; iters {int(it[i, w])}, alive/iter "
              f"{alive[i, w] / max(it[i, w], 1):.1f}; clocks fill {int(fill[i, w])} hit {int(hit[i, w])} "
              f"hard {int(hard[i, w])} soft {int(soft[i, w])} light-rest {int(light[i, w] - hard[i, w] - soft[i, w])} "
              f"scat {int(scat[i, w])}; coop {int(coop[i, w])} seq {int(seq[i, w])}; wave us {end[i, w] - start[i, w]:.0f}"
              f" start {start[i, w]:.0f}")
for i in order[:4]:
    # slots 16..31: s_memrealtime at every 4th shade iteration, unless the
    # workgroup ran a lone path (slot 42 != 0): then the kernel stores the lone
    # path's section clocks there instead (rt_kernel.hip, RT_WG_TIMING epilogue)
    if d[i, 0, 42] != 0:
        print(f"    WG {int(i)} ran a lone path ({int(d[i, 0, 42])} bounces): its section clocks",
              [int(v) for v in d[i, 0, 16:32]])
        continue
    ts = [(int(v) - t0) / 100.0 for v in d[i, 0, 17:32] if v != 0]
    print(f"    WG {int(i)} time at every 4th shade iteration (us):", [round(t, 1) for t in ts])
late = end.max(axis=1) > 0.7 * span
print(f"  WGs ending after 70% of the span: {int(late.sum())}; of them split {int((d[late, 0, 14] > 0).sum())}, "
      f"mean iters {it[late].mean():.0f}, mean start {start[late].mean():.0f} us")
solo = d[:, 0, 42] != 0  # lone-path bounces (slot 42) / entries into solo_path (slot 43)
print(f"  WGs that ran a lone path (solo_path): {int(solo.sum())} of {nwg}; entries {int(d[:, 0, 43].sum())}, "
      f"lone-path bounces {int(d[:, 0, 42].sum())}")
busy = dur.sum()
print(f"  mean waves in flight {busy / span:.1f}")
bclk = d[:, 0, 32:37].astype(np.float64)
bcnt = d[:, 0, 37:42].astype(np.float64)
names = ["1", "2", "3-4", "5-8", ">8"]
for label, sel in (("all WGs", np.ones(nwg, bool)), ("WGs ending after 70% of the span", late)):
    c, n = bclk[sel].sum(axis=0), bcnt[sel].sum(axis=0)
    print(f"  {label}: shade iterations by live lanes " + ", ".join(
        f"{names[i]}: {int(n[i])} it {c[i] / max(c.sum(), 1):.0%} clk ({c[i] / max(n[i], 1):.0f}/it)" for i in range(5)))
