#!/usr/bin/env python3
"""Procedural 10k-sphere scene for configs C4/C5 (BASELINE.json configs[3..4]).

The reference has no scene generator, so the build defines one
(SURVEY.md §8d).  Random source: the reference's own FastRandom xorshift64*
(internal/math/advanced_math.go:7-24), seeded 42, Float64 = Next()/(2^64-1).
Per sphere, draws in this order: x, y, z, radius, material selector, then the
material's parameters:
  centre x in [-30,30], y in [-20,20], z in [-80,-10]; radius in [0.3,1.0];
  selector < 0.4 metal (colour U[0.5,1]^3, roughness U[0,0.3]),
           < 0.7 glass (colour U[0.7,1]^3, refractionIndex 1.5),
           else  lambertian (colour U[0.2,0.9]^3).
Camera at the origin (the reference camera looks down -Z), aspect 1.78; two
point lights.  Output is canonical JSON (sorted keys, repr floats), so its
SHA-256 is stable: see EXPECTED_SHA256 (checked by tests/test_scenes.py).

usage: gen_spheres.py [N] [out.json]
"""
import hashlib
import json
import sys

EXPECTED_SHA256 = {10000: "6a6ca961749f916cc4abab84a8268e2c71b661f98dd9d43a0454ff38de3f6cea"}

MASK = (1 << 64) - 1


class FastRandom:
    def __init__(self, seed):
        self.state = seed & MASK

    def next(self):
        s = self.state
        s ^= s >> 12
        s ^= (s << 25) & MASK
        s ^= s >> 27
        self.state = s
        return (s * 2685821657736338717) & MASK

    def float64(self):
        return float(self.next()) / float(MASK)

    def range(self, lo, hi):
        return lo + self.float64() * (hi - lo)


def generate(n=10000, seed=42):
    r = FastRandom(seed)
    objects = []
    for _ in range(n):
        x = r.range(-30.0, 30.0)
        y = r.range(-20.0, 20.0)
        z = r.range(-80.0, -10.0)
        rad = r.range(0.3, 1.0)
        sel = r.float64()
        if sel < 0.4:
            mat = {
                "type": "metal",
                "color": [r.range(0.5, 1.0), r.range(0.5, 1.0), r.range(0.5, 1.0)],
                "roughness": r.range(0.0, 0.3),
            }
        elif sel < 0.7:
            mat = {
                "type": "glass",
                "color": [r.range(0.7, 1.0), r.range(0.7, 1.0), r.range(0.7, 1.0)],
                "refractionIndex": 1.5,
            }
        else:
            mat = {"type": "lambertian", "color": [r.range(0.2, 0.9), r.range(0.2, 0.9), r.range(0.2, 0.9)]}
        objects.append({"type": "sphere", "position": [x, y, z], "radius": rad, "material": mat})
    return {
        "camera": {"position": [0, 0, 0], "lookAt": [0, 0, -1], "up": [0, 1, 0], "fov": 60, "aspectRatio": 1.78},
        "objects": objects,
        "lights": [
            {"type": "point", "position": [20, 40, 10], "color": [1, 1, 1], "intensity": 3000.0},
            {"type": "point", "position": [-30, 20, -20], "color": [1, 0.9, 0.8], "intensity": 1500.0},
        ],
    }


def dumps(scene):
    return json.dumps(scene, sort_keys=True, separators=(",", ":"))


def sha256(text):
    return hashlib.sha256(text.encode()).hexdigest()


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    out = sys.argv[2] if len(sys.argv) > 2 else f"spheres{n}.json"
    text = dumps(generate(n))
    with open(out, "w") as f:
        f.write(text)
    print(out, sha256(text))
