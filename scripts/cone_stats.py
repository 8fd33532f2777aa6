#!/usr/bin/env python3
"""How much of C4's soft-shadow work a shadow-cone test can settle (dev
probe, CPU/numpy, no GPU): primary hits of the 10k-sphere scene
(scenes/gen_spheres.py) at random pixels of 1920x1080, both lights; for each
(hit, light) whose hard ray is clear, the spheres the cone of half-angle
asin(0.1) toward the light can meet (the test of rt_wavefront.hip wf_cone,
hit sphere excluded by the same rule), and the BVH nodes a cone walk visits
against what 16 soft rays' any-hit walks visit (a median-split BVH with
4-sphere leaves, node bounding balls for the cone).

usage: cone_stats.py [pixels]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scenes"))


def main():
    import gen_spheres

    npix = int(sys.argv[1]) if len(sys.argv) > 1 else 600
    sc = gen_spheres.generate(10000)
    C = np.array([o["position"] for o in sc["objects"]], float)
    R = np.array([o["radius"] for o in sc["objects"]], float)
    lights = [np.array(l["position"], float) for l in sc["lights"]]

    nodes = []  # (lo, hi, left, right, spheres)

    def build(idx):
        lo, hi = (C[idx] - R[idx, None]).min(0), (C[idx] + R[idx, None]).max(0)
        k = len(nodes)
        nodes.append(None)
        if len(idx) <= 4:
            nodes[k] = (lo, hi, -1, -1, idx)
            return k
        cl = C[idx]
        ax = np.argmax(cl.max(0) - cl.min(0))
        s = idx[np.argsort(cl[:, ax])]
        m = len(s) // 2
        left, right = build(s[:m]), build(s[m:])
        nodes[k] = (lo, hi, left, right, None)
        return k

    build(np.arange(len(C)))
    LO = np.array([n[0] for n in nodes])
    HI = np.array([n[1] for n in nodes])
    BC, BR = (LO + HI) / 2, np.linalg.norm(HI - LO, axis=1) / 2

    def in_cone(c, r, P, u, dist):
        v = c - P
        dc = np.linalg.norm(v)
        ra = r * 1.00001 + 1e-5 * dc
        if dc <= ra:
            return True
        if dc - ra > dist:
            return False
        return v @ u >= 0.99498 * np.sqrt(max(dc * dc - ra * ra, 0)) - 0.1 * ra - 1e-5 * dc

    def sph_hit(i, o, d, tmax):
        oc = o - C[i]
        hb, c = oc @ d, oc @ oc - R[i] ** 2
        disc = hb * hb - c
        if disc < 0:
            return False
        s = np.sqrt(disc)
        return 0.001 < -hb - s < tmax or 0.001 < -hb + s < tmax

    def box_hit(k, o, inv, tmax):
        t0, t1 = (LO[k] - o) * inv, (HI[k] - o) * inv
        return max(np.minimum(t0, t1).max(), 0.001) <= min(np.maximum(t0, t1).min(), tmax)

    def ray_any(o, d, tmax):
        inv, st, vis = 1 / d, [0], 0
        while st:
            k = st.pop()
            vis += 1
            if not box_hit(k, o, inv, tmax):
                continue
            n = nodes[k]
            if n[2] < 0:
                if any(sph_hit(i, o, d, tmax) for i in n[4]):
                    return True, vis
            else:
                st += [n[3], n[2]]
        return False, vis

    def cone_all(P, u, dist, excl):
        st, vis, cand = [0], 0, []
        while st:
            k = st.pop()
            vis += 1
            if not in_cone(BC[k], BR[k], P, u, dist):
                continue
            n = nodes[k]
            if n[2] < 0:
                cand += [i for i in n[4] if i != excl and in_cone(C[i], R[i], P, u, dist)]
            else:
                st += [n[3], n[2]]
        return cand, vis

    rng = np.random.default_rng(3)
    W, H, aspect = 1920, 1080, 1.78
    cands, cone_vis, soft_vis = [], [], []
    for _ in range(npix):
        x, y = rng.uniform(0, W), rng.uniform(0, H)
        d = np.array([-aspect + x / W * 2 * aspect, -1 + 2 * y / H, -1.0])
        oc = -C
        a, hb, c = d @ d, oc @ d, (oc * oc).sum(1) - R * R
        disc = hb * hb - a * c
        ok = disc >= 0
        t1 = (-hb - np.sqrt(np.where(ok, disc, 0))) / a
        t = np.where(ok & (t1 > 0.001), t1, np.inf)
        i = int(np.argmin(t))
        if not np.isfinite(t[i]):
            continue
        P = d * t[i]
        N = (P - C[i]) / R[i]
        for L in lights:
            lv = L - P
            dist = np.linalg.norm(lv)
            u = lv / dist
            if ray_any(P, u, dist)[0]:
                continue
            cc, v = cone_all(P, u, dist, i if N @ u >= 0.1015 else -1)
            cands.append(len(cc))
            cone_vis.append(v)
            sv = 0
            for _s in range(16):
                while True:
                    p = rng.uniform(-1, 1, 3)
                    if p @ p < 1:
                        break
                dd = u + 0.1 * p
                sv += ray_any(P, dd / np.linalg.norm(dd), dist)[1]
            soft_vis.append(sv)
    cands, cone_vis, soft_vis = map(np.array, (cands, cone_vis, soft_vis))
    over = cands > 16
    out = {
        "clear_cones": int(len(cands)),
        "empty_fraction": round(float((cands == 0).mean()), 4),
        "candidates_mean": round(float(cands.mean()), 3),
        "candidates_p50_p90_p99_max": [float(x) for x in np.percentile(cands, [50, 90, 99])] + [int(cands.max())],
        "more_than_16": round(float(over.mean()), 4),
        "more_than_32_64_128": [round(float((cands > k).mean()), 4) for k in (32, 64, 128)],
        "cone_walk_nodes_mean": round(float(cone_vis.mean()), 1),
        "soft_rays_nodes_mean_per_cone": round(float(soft_vis.mean()), 1),
        "nodes_with_lists_vs_rays": round(float((cone_vis.sum() + soft_vis[over].sum()) / soft_vis.sum()), 4),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
