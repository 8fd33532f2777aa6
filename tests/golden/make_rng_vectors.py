#!/usr/bin/env python3
"""Writes tests/golden/rng_v4.json: known-answer vectors of the random stream
spec v4 (include/rt_rng.h): the per-sample stream (unchanged since v3) and
v4's soft-shadow streams, computed by an independent pure-Python statement of
the spec (tests/rng_spec.py).  Regenerate only when the spec changes."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from rng_spec import draws, soft_draws, soft_points  # noqa: E402

KEYS = [(1, 0, 0), (1, 123456, 99), (42, 479999, 0), (0xDEADBEEFCAFEF00D, 2**32 - 1, 2**32 - 1)]

out = []
for seed, pixel, sample in KEYS:
    raw, vals = draws(seed, pixel, sample, 12)
    out.append({"seed": seed, "pixel": pixel, "sample": sample, "raw": raw, "draws": [v.hex() for v in vals]})
SOFT_KEYS = [(1, 0, 0, 0, 0), (1, 123456, 99, 3, 1), (42, 479999, 0, 49, 2), (7, 2**32 - 1, 2**24, 0, 31)]
soft = []
for seed, pixel, sample, depth, light in SOFT_KEYS:
    pts, tries = soft_points(seed, pixel, sample, depth, light)
    soft.append({"seed": seed, "pixel": pixel, "sample": sample, "depth": depth, "light": light,
                 "raw": soft_draws(seed, pixel, sample, depth, light, 12), "tries": tries,
                 "points": [[c.hex() for c in p] for p in pts]})
with open(os.path.join(HERE, "rng_v4.json"), "w") as f:
    json.dump({"spec": "rt_rng.h v4 (PCG-XSH-RR 64/32, SplitMix64-keyed; soft-shadow streams per (sample, depth, "
                       "light))", "vectors": out, "soft_vectors": soft}, f, indent=1)
print("wrote", len(out), "vectors and", len(soft), "soft-stream vectors")
