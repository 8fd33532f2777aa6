#!/usr/bin/env python3
"""Oracle fixtures for the 10k-sphere configs C4 and C5 (BASELINE.json
configs[3], configs[4]) at their FULL resolution, on a sample of tiles.

The linear-scan oracle (oracle/oracle.c, the restatement of hitWorld's
10,000-sphere scan, renderer.go:333-346) cannot render a whole C4/C5 frame in
reasonable time (~10^13 sphere tests), but it renders ONE 32x32 tile at full
spp in about a minute on one core: tile t alone is `oracle_render(rank=t,
world=ntiles, max_tiles=1)`, and since the random stream is keyed by the
global (pixel, sample) the tile is the same tile the full frame holds.

  survey  -- per-tile path counts at 1 spp on every STRIDE-th tile (oracle),
             to find the tiles with the longest paths (the heaviest tiles);
  render  -- the chosen tiles at full spp and depth 50: linear float32 and
             RGBA8 per tile, plus the oracle's path counts, into
             tests/golden/oracle_c4_tiles.npz / oracle_c5_tiles.npz.

The GPU tests (tests/test_gpu_bvh_tiles.py) render the whole C4 frame and the
packed shares of C5 ranks 0 and 7 of 8 and compare these tiles bit for bit.
Run once (a few CPU-minutes per tile; tiles run in parallel threads):
    python tests/golden/make_bvh_tiles.py survey c4 4
    python tests/golden/make_bvh_tiles.py survey c5 64 0 7    (ranks 0 and 7 of 8)
    python tests/golden/make_bvh_tiles.py render c4 <tile> <tile> ...
The wider sample (r06; tests/test_gpu_bvh_tiles.py checks both):
    SUFFIX=_more python tests/golden/make_bvh_tiles.py render c4 <12 tiles of survey_c4.json, spread over its ranking>
    SUFFIX=_more python tests/golden/make_bvh_tiles.py survey c5 64 19 45    (ranks 3 and 5 of 8)
    SUFFIX=_more python tests/golden/make_bvh_tiles.py render c5 <2 tiles of rank 3, 2 of rank 5>
"""
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd"), os.path.dirname(HERE)):
    sys.path.insert(0, p)
import oracle  # noqa: E402
import rtgo  # noqa: E402
from scene_cases import make_settings, spheres10k_scene  # noqa: E402

# SUFFIX=_more: write survey_<cfg>_more.json / oracle_<cfg>_tiles_more.npz (the
# second, wider sample of tiles) instead of the first files
SUFFIX = os.environ.get("SUFFIX", "")
# (width, height, spp) of each config; depth 50, soft shadows, recursion (defaults)
CONFIGS = {"c4": (1920, 1080, 64), "c5": (3840, 2160, 256)}


def render_tile(scene, w, h, st, t):
    """Tile t alone (oracle threads = 1): (linear (32,32,3) f64, rgba (32,32,4), counts)."""
    tx_n = (w + 31) // 32
    n = rtgo.num_tiles(w, h)
    lin, rgba, counts = oracle.render(scene, w, h, st, rank=t, world=n, nthreads=1, max_tiles=1, counts=True)
    tx, ty = t % tx_n, t // tx_n
    x0, y0 = tx * 32, ty * 32
    return lin[y0:y0 + 32, x0:x0 + 32], rgba[y0:y0 + 32, x0:x0 + 32], counts


def survey(cfg, stride, offsets, workers):
    w, h, _ = CONFIGS[cfg]
    scene = spheres10k_scene(rtgo)
    st = make_settings(rtgo, {"samples": 1}, seed=1)
    tiles = sorted(t for o in offsets for t in range(o, rtgo.num_tiles(w, h), stride))
    t0 = time.time()
    with ThreadPoolExecutor(workers) as ex:
        res = list(ex.map(lambda t: render_tile(scene, w, h, st, t)[2], tiles))
    out = {str(t): c for t, c in zip(tiles, res)}
    path = os.path.join(HERE, f"survey_{cfg}{SUFFIX}.json")
    with open(path, "w") as f:
        json.dump(out, f)
    top = sorted(tiles, key=lambda t: -out[str(t)]["bounce_rays"])[:12]
    print(f"{path}: {len(tiles)} tiles in {time.time() - t0:.0f} s; heaviest (bounce rays at 1 spp):")
    for t in top:
        print(f"  tile {t}: {out[str(t)]['bounce_rays']} bounce rays, {out[str(t)]['shadow_rays']} shadow rays")


def render(cfg, tiles, workers):
    w, h, spp = CONFIGS[cfg]
    scene = spheres10k_scene(rtgo)
    st = make_settings(rtgo, {"samples": spp}, seed=1)
    t0 = time.time()
    with ThreadPoolExecutor(workers) as ex:
        res = list(ex.map(lambda t: render_tile(scene, w, h, st, t), tiles))
    lin = np.stack([r[0] for r in res]).astype(np.float32)
    rgba = np.stack([r[1] for r in res])
    counts = np.array([[r[2][k] for k in rtgo.COUNT_FIELDS] for r in res], np.uint64)
    assert not np.isnan(lin).any()
    path = os.path.join(HERE, f"oracle_{cfg}_tiles{SUFFIX}.npz")
    np.savez_compressed(path, tiles=np.array(tiles, np.int32), linear=lin, rgba=rgba, counts=counts,
                        config=np.array([w, h, spp, 50, 1], np.int32))
    print(f"{path}: tiles {tiles} at {w}x{h}x{spp} in {time.time() - t0:.0f} s, {os.path.getsize(path)} B")


if __name__ == "__main__":
    mode, cfg = sys.argv[1], sys.argv[2]
    workers = int(os.environ.get("WORKERS", str(os.cpu_count() or 1)))
    if mode == "survey":
        # survey <cfg> <stride> [offset ...]: tiles offset + k * stride
        survey(cfg, int(sys.argv[3]) if len(sys.argv) > 3 else 8, [int(o) for o in sys.argv[4:]] or [0], workers)
    else:
        render(cfg, [int(t) for t in sys.argv[3:]], workers)
