#!/usr/bin/env python3
"""Where a one-shot render's time goes (dev probe): rt_render (device state
created and freed every call, like one `raytracer` process per frame) on the
headline frame, with rt_stats' breakdown (create, scene, launch, kernels +
download, destroy), medians over N calls after one warm-up; then the
`raytracer` CLI as a fresh process on the same frame (HIP start-up
included), whose benchmark_data.json is written to gpurun_out/cli_c2/.

usage: oneshot_probe.py [N]
"""
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "concurrent-raytracer-go_amd")]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    out = {}
    # the CLI first, in a fresh process (nothing of this one's HIP state)
    exe = os.path.join(ROOT, "concurrent-raytracer-go_amd", "build", "raytracer")
    scene = os.path.join(ROOT, "scenes", "sphere_reflections_light_facing.json")
    od = os.path.join(ROOT, "gpurun_out", "cli_c2")
    os.makedirs(od, exist_ok=True)
    t0 = time.perf_counter()
    p = subprocess.run([exe, scene, os.path.join(od, "out.png"), "800", "600"], capture_output=True, text=True,
                       timeout=300)
    wall = time.perf_counter() - t0
    bd = json.load(open(os.path.join(od, "benchmark_data.json"))) if p.returncode == 0 else None
    out["cli"] = {"rc": p.returncode, "process_wall_s": round(wall, 4), "benchmark_data": bd,
                  "stdout_tail": p.stdout[-400:]}
    import rtgo

    sc = rtgo.Scene.load_from_file(scene)
    st = rtgo.default_settings()
    rows = []
    for i in range(n + 1):
        st.seed = 1 + i
        _, _, s = rtgo.render(sc, 800, 600, st)
        if i:
            rows.append({k: getattr(s, k) for k in ("render_seconds", "create_seconds", "scene_seconds",
                                                     "launch_seconds", "download_seconds", "destroy_seconds",
                                                     "kernel_seconds")})
    out["oneshot_median_ms"] = {k: round(statistics.median(r[k] for r in rows) * 1e3, 4) for k in rows[0]}
    r = rtgo.ParallelRenderer()
    r.settings = rtgo.default_settings()
    rows = []
    for i in range(n + 1):
        r.settings.seed = 1 + i
        r.render(sc, 800, 600)
        s = r.last_stats
        if i:
            rows.append({k: getattr(s, k) for k in ("render_seconds", "scene_seconds", "launch_seconds",
                                                     "download_seconds", "kernel_seconds")})
    r.close()
    out["persistent_median_ms"] = {k: round(statistics.median(x[k] for x in rows) * 1e3, 4) for k in rows[0]}
    print(json.dumps(out, indent=1))
    with open(os.path.join(ROOT, "gpurun_out", "oneshot_probe.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
