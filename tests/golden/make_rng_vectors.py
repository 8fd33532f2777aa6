#!/usr/bin/env python3
"""Writes tests/golden/rng_v3.json: known-answer vectors of the random stream
spec v3 (include/rt_rng.h), computed by an independent pure-Python statement
of the spec (tests/rng_spec.py).  Regenerate only when the spec changes."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from rng_spec import draws  # noqa: E402

KEYS = [(1, 0, 0), (1, 123456, 99), (42, 479999, 0), (0xDEADBEEFCAFEF00D, 2**32 - 1, 2**32 - 1)]

out = []
for seed, pixel, sample in KEYS:
    raw, vals = draws(seed, pixel, sample, 12)
    out.append({"seed": seed, "pixel": pixel, "sample": sample, "raw": raw, "draws": [v.hex() for v in vals]})
with open(os.path.join(HERE, "rng_v3.json"), "w") as f:
    json.dump({"spec": "rt_rng.h v3 (PCG-XSH-RR 64/32, SplitMix64-keyed)", "vectors": out}, f, indent=1)
print("wrote", len(out), "vectors")
