#!/usr/bin/env python3
"""Writes tests/golden/oracle_*.npz: small whole-image fixtures rendered by
the CPU oracle (oracle/oracle.c) with the random stream spec v4 (regenerated in round 5 for v4).

These are SELF-PINS of this build (the reference has no renderer goldens and
no Go toolchain exists here — SURVEY.md §4, §8c): they freeze the oracle's
output so any later change to the oracle or the kernel that alters an image
is caught, and the GPU parity tests compare the kernel with them bit for bit.
Regenerate only with a deliberate spec change:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd"), os.path.dirname(HERE)):
    sys.path.insert(0, p)
import oracle  # noqa: E402
import rtgo  # noqa: E402
from scene_cases import GOLDEN_CASES, load_case, make_settings  # noqa: E402


def main():
    for name, loader, w, h, over, seed in GOLDEN_CASES:
        scene = load_case(rtgo, loader)
        st = make_settings(rtgo, over, seed)
        lin, rgba, counts = oracle.render(scene, w, h, st, counts=True)
        path = os.path.join(HERE, f"oracle_{name}.npz")
        np.savez_compressed(path, linear=lin, rgba=rgba, counts=np.array([counts[k] for k in rtgo.COUNT_FIELDS],
                                                                           np.uint64))
        print(f"{path}: {w}x{h} {over} seed {seed}; mean {np.nanmean(lin):.6f}, {os.path.getsize(path)} B")


if __name__ == "__main__":
    main()
