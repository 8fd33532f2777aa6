"""GPU: no kernel reads another lane's value from an inactive lane.

__shfl (ds_bpermute) from a lane that is inactive at the read returns no
data.  Owner-state reads therefore belong in converged code; a rejected r03
soft-shadow variant hung because it read an owner's jump coefficients inside
an owner-only branch.  The checking build
(concurrent-raytracer-go_amd/build/xlane/librtgo.so, `make xlane`,
-DRT_CHECK_XLANE in csrc/rt_device.h) counts every such read.  This test
renders scenes that reach every cross-lane form of the kernels (solo paths,
wide mode, soft_queue with its cooperative tail, soft_coop, split pixels,
the wavefront path) with that build, in a child process, and requires zero.
The checking build also compiles in the lone-path form (RT_SOLO=1, off in the
product since r05), which the 50-bounce mirror probe and the
every-pixel-split render reach; their radiance must equal the product's
bit for bit (which the other GPU tests hold to the oracle).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
XLIB = os.path.join(ROOT, "concurrent-raytracer-go_amd", "build", "xlane", "librtgo.so")

JOBS = r"""
import hashlib, json
import rtgo
from scene_cases import CUBE_SCENES, load_case, make_settings
from test_gpu_paths import _sphere_field

def render_jobs(facing):
    jobs = [
        (rtgo.Scene.load_from_file(facing), 160, 120, {"samples": 24}, None),
        (load_case(rtgo, ("json", None)), 96, 64, {"samples": 16}, None),
        (load_case(rtgo, ("json", None)), 64, 48, {"samples": 40, "max_depth": 12}, {"block_work": 1}),
        (rtgo.Scene.from_json_text(json.dumps(CUBE_SCENES["mirror_probe_glass_cube"])), 48, 32, {"samples": 8}, None),
        (rtgo.Scene.from_json_text(json.dumps(_sphere_field(300, seed=5))), 64, 48, {"samples": 4}, None),
    ]
    hashes = []
    for scene, w, h, over, tun in jobs:
        r = rtgo.ParallelRenderer()
        r.settings = make_settings(rtgo, over, 3)
        if tun:
            r.set_tuning(rtgo.default_tuning(**tun))
        r.render(scene, w, h)
        hashes.append(hashlib.sha1(r.last_linear.tobytes()).hexdigest())
        r.close()
    return hashes
"""

CHILD = r"""
import json, sys
sys.path[:0] = [%(tests)r, %(pkg)r]
import ctypes
exec(%(jobs)r)
lib = rtgo.lib()
out = ctypes.c_uint64(0)
assert lib.rt_debug_xlane_faults(0, 1, ctypes.byref(out)) == 0, lib.rt_last_error()
hashes = render_jobs(%(facing)r)
assert lib.rt_debug_xlane_faults(0, 0, ctypes.byref(out)) == 0, lib.rt_last_error()
print("XLANE_FAULTS", out.value)
print("HASHES", json.dumps(hashes))
"""


@pytest.mark.skipif(not os.path.exists(XLIB), reason="build/xlane/librtgo.so not built (make xlane)")
def test_no_cross_lane_read_from_an_inactive_lane():
    facing = os.path.join(ROOT, "scenes", "sphere_reflections_light_facing.json")
    code = CHILD % {"tests": os.path.join(ROOT, "tests"), "pkg": os.path.join(ROOT, "concurrent-raytracer-go_amd"),
                    "jobs": JOBS, "facing": facing}
    env = dict(os.environ, RTGO_LIB=XLIB)
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    print(p.stdout[-2000:], p.stderr[-2000:])
    assert p.returncode == 0, p.stderr[-2000:]
    faults = int(p.stdout.split("XLANE_FAULTS")[1].split()[0])
    assert faults == 0, faults
    # the same renders on the product library (lone-path form off)
    child = json.loads(p.stdout.split("HASHES")[1].strip().splitlines()[0])
    ns = {}
    exec(JOBS, ns)
    assert ns["render_jobs"](facing) == child
