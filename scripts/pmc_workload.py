#!/usr/bin/env python3
"""The bench workload alone (no counting variant, no second scene): K renders
of one bench config (PMC_CONFIG: c2 default, c2_committed, c3, c4, c5; the
scenes and sizes of bench.py CONFIGS) on one GPU, one frame per launch.  Run
under rocprofv3 --pmc by scripts/profile.sh so each PMC pass sees only the
config's kernels.  PMC_SIZE=W,H,SPP overrides the size (the instruction-mix
passes of scripts/profile_instmix.sh use C4's scene at 960x540x16).
PMC_FRAMES=B (c2/c3): K launches of B frames each (rt_context_render_frames_async,
the bench's timed launches) instead of K one-frame launches."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import rtgo  # noqa: E402
from bench import CONFIGS, load_scene  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
cfg = os.environ.get("PMC_CONFIG", "c2")
if os.environ.get("PMC_SCENE") == "spheres10k":  # (older spelling: C4's scene)
    cfg = "c4"
elif os.environ.get("PMC_SCENE") == "committed":
    cfg = "c2_committed"
spec, W, H, SPP = CONFIGS[cfg][:4]
if os.environ.get("PMC_SIZE"):
    W, H, SPP = (int(v) for v in os.environ["PMC_SIZE"].split(","))
st = rtgo.default_settings()
st.samples = SPP
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
ctx = rtgo.Context(0)
ctx.set_scene(load_scene(rtgo, spec))
B = int(os.environ.get("PMC_FRAMES", "1"))
lin = torch.zeros((B, W * H * 3), dtype=torch.float32, device="cuda")
rgba = torch.zeros((B, W * H * 4), dtype=torch.uint8, device="cuda")
for i in range(K):
    if B == 1:
        st.seed = 1 + i
        ctx.render_async(W, H, st, lin[0].data_ptr(), rgba[0].data_ptr(), s.cuda_stream)
    else:
        ctx.render_frames_async(W, H, st, [1 + i * B + f for f in range(B)], [lin[f].data_ptr() for f in range(B)],
                                [rgba[f].data_ptr() for f in range(B)], s.cuda_stream)
torch.cuda.synchronize()
print("rendered", K, "launches of", B, "frames of", cfg, f"{W}x{H}x{SPP}; linear sum", float(lin.double().sum()))
