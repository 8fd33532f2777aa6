#!/usr/bin/env python3
"""Where the headline frame's long paths are (dev analysis, CPU only).

Uses the oracle's per-sample path lengths (oracle.path_lengths: traceRay
calls per sample, renderer.go:165-227) of the headline frame (800x600x100,
depth 50, the facing scene) at three seeds, and asks whether a pilot render
could have found the pixels that hold the long paths:
  - the path-length histogram and the pixels with a >= 40-bounce path;
  - how many of those pixels recur across seeds;
  - the one-sample pilot's neighbourhood estimate of them (sched_est);
  - how many a K-sample pilot (any path of >= 3 bounces) would flag / catch.
usage: scripts/path_stats.py [out.json]   (~3 s per seed on 8 cores)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd")]

import oracle  # noqa: E402
import rtgo  # noqa: E402


def nbmax(a):
    m = a.copy()
    m[1:, :] = np.maximum(m[1:, :], a[:-1, :])
    m[:-1, :] = np.maximum(m[:-1, :], a[1:, :])
    m[:, 1:] = np.maximum(m[:, 1:], a[:, :-1])
    m[:, :-1] = np.maximum(m[:, :-1], a[:, 1:])
    return m


def main():
    scene = rtgo.Scene.load_from_file(os.path.join(ROOT, "scenes", "sphere_reflections_light_facing.json"))
    L = {}
    for seed in (1, 2, 3):
        st = rtgo.default_settings()
        st.samples, st.seed = 100, seed
        L[seed] = oracle.path_lengths(scene, 800, 600, st).astype(np.int32)
    out = {"frame": "sphere_reflections_light_facing 800x600x100 depth 50", "seeds": [1, 2, 3]}
    h = np.bincount(L[1].ravel(), minlength=52)
    out["histogram_seed1"] = {int(k): int(v) for k, v in enumerate(h) if v}
    long_px = {s: (L[s] >= 40).any(-1) for s in L}
    out["pixels_with_40_bounce_path"] = {s: int(long_px[s].sum()) for s in L}
    out["common_seed1_seed2"] = int((long_px[1] & long_px[2]).sum())
    out["union_three_seeds"] = int((long_px[1] | long_px[2] | long_px[3]).sum())
    allL = np.concatenate([L[1], L[2], L[3]], -1)
    p = (allL >= 40).mean(-1)
    out["per_sample_probability_quantiles"] = [float(x) for x in np.quantile(p[p > 0], [0.1, 0.5, 0.9])]
    # the one-sample pilot (sample 0 of seed 1, paths cut at 12 bounces) and
    # sched_est's neighbourhood maximum, against the long paths of seeds 2, 3
    est = nbmax(np.minimum(L[1][:, :, 0], 12))
    out["pilot_estimate_of_long_path_pixels"] = {
        s: {int(k): int(v) for k, v in enumerate(np.bincount(est[long_px[s]], minlength=13)) if v} for s in (2, 3)}
    split = 100 * (est + 0.02) > 384
    out["pixels_split_by_pilot"] = int(split.sum())
    out["long_path_pixels_split"] = {s: round(float((long_px[s] & split).sum() / long_px[s].sum()), 3) for s in (2, 3)}
    kp = {}
    for K in (4, 8, 16, 32):
        flagged = (L[1][:, :, :K] >= 3).any(-1)
        kp[K] = {"flagged": int(flagged.sum()),
                 "caught": [round(float((long_px[s] & flagged).sum() / long_px[s].sum()), 3) for s in (2, 3)]}
    out["k_sample_pilot_any_3_bounce_path"] = kp
    out["live_pixels"] = int((L[1].max(-1) >= 2).sum())
    text = json.dumps(out, indent=1)
    print(text)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
