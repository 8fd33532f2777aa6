#!/usr/bin/env python3
"""Calibration workload for the WRITE_SIZE / FETCH_SIZE counters (dev tool).

MI355X_MICROARCH.md calibrates WRITE_SIZE only for 16-B-per-lane stores; the
render kernel's epilogue writes a pixel as one 12-B float3 store plus one
4-B RGBA8 store per lane.  unpack_kernel (rt_kernel.hip) writes exactly that
pattern, one thread per image pixel, fully coalesced: W*H*16 bytes per
launch, and reads the same 16 B per pixel from the packed share.  Run under
rocprofv3 --pmc WRITE_SIZE (and FETCH_SIZE) by scripts/profile.sh; the
counter / known-bytes ratio corrects the render kernel's traffic figure.
usage: pmc_calib.py [K]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd")]
import torch  # noqa: E402

import rtgo  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
W, H = 3840, 2160
nb = rtgo.packed_bytes(W, H, 1)
g = torch.ones(nb, dtype=torch.uint8, device="cuda")
lin = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
rgba = torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
for _ in range(K):
    rtgo.unpack_tiles_async(W, H, 1, g.data_ptr(), lin.data_ptr(), rgba.data_ptr(), 0)
torch.cuda.synchronize()
print(f"unpacked {K} x {W}x{H}: {W * H * 16} B written per launch, {nb} B share")
