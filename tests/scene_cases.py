"""Scenes used by the parity tests (shared by CPU and GPU tests)."""
import json
import os

SCENES = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scenes")

# Every JSON-reachable material (scene.go:104-148), spheres and a cube, a
# light behind the camera side, facing the reference's fixed -Z camera.
ALL_MATERIALS = {
    "camera": {"position": [0, 0.5, 6], "lookAt": [0, 0, 0], "up": [0, 1, 0], "fov": 60, "aspectRatio": 1.5},
    "objects": [
        {"type": "sphere", "position": [0, -1001, 0], "radius": 1000,
         "material": {"type": "lambertian", "color": [0.5, 0.5, 0.5]}},
        {"type": "sphere", "position": [-3.2, 0, 0], "radius": 0.8,
         "material": {"type": "metal", "color": [0.9, 0.6, 0.3], "roughness": 0.2, "metallic": 0.85,
                      "specular": 0.7}},
        {"type": "sphere", "position": [-1.4, 0, 0.5], "radius": 0.7,
         "material": {"type": "glass", "color": [0.9, 0.95, 1.0], "refractionIndex": 1.5}},
        {"type": "sphere", "position": [0.3, 0, 0], "radius": 0.8,
         "material": {"type": "dielectric", "refractionIndex": 1.33}},
        {"type": "sphere", "position": [2.0, 0, -0.5], "radius": 0.8,
         "material": {"type": "shiny", "color": [0.2, 0.8, 0.3], "roughness": 0.1, "metallic": 0.6,
                      "specular": 0.5}},
        {"type": "sphere", "position": [3.6, 0.2, 0], "radius": 0.7,
         "material": {"type": "perfectmirror", "color": [0.8, 0.8, 0.8], "roughness": 0.05}},
        {"type": "sphere", "position": [0, 2.2, -2], "radius": 0.6,
         "material": {"type": "diffuselight", "color": [4, 4, 3.5]}},
        {"type": "cube", "position": [1.2, -0.6, 1.6], "size": [0.8, 0.8, 0.8],
         "material": {"type": "metal", "color": [0.7, 0.7, 0.9], "roughness": 0.0, "metallic": 1.0}},
        {"type": "cube", "position": [-2.2, -0.7, 2.0], "size": [0.6, 0.6, 0.6],
         "material": {"type": "lambertian", "color": [0.8, 0.1, 0.1]}},
        {"type": "sphere", "position": [-0.5, -0.75, 2.2], "radius": 0.25,
         "material": {"type": "metal", "color": [0.95, 0.95, 0.95], "roughness": 0.6, "metallic": 0.55}},
        {"type": "sphere", "position": [0.9, 1.0, 1.0], "radius": 0.3,
         "material": {"type": "unknownkind", "color": [0.3, 0.3, 0.9]}},
    ],
    "lights": [
        {"type": "point", "position": [4, 6, 6], "color": [1, 1, 1], "intensity": 40.0},
        {"type": "point", "position": [-5, 3, 4], "color": [0.8, 0.8, 1], "intensity": 20.0},
        {"type": "point", "position": [0, 0.5, 0.3], "color": [1, 0.5, 0.5], "intensity": 0.5},
    ],
}


def scene_path(name):
    return os.path.join(SCENES, name)


def all_materials_json():
    return json.dumps(ALL_MATERIALS)


# (id, loader, width, height, settings overrides)
PARITY_CASES = [
    ("spheres_facing", ("file", "sphere_reflections_light_facing.json"), 96, 72, {"samples": 8}),
    ("spheres_as_committed", ("file", "sphere_reflections_light.json"), 64, 48, {"samples": 4}),
    ("silver_facing", ("file", "final_silver_prism_purple_cube_facing.json"), 96, 72, {"samples": 6}),
    ("all_materials", ("json", None), 96, 64, {"samples": 8}),
    ("all_materials_hard_shadows", ("json", None), 64, 48, {"samples": 4, "soft_shadows": 0}),
    ("all_materials_no_recursion", ("json", None), 64, 48, {"samples": 4, "recursive_reflections": 0}),
    ("all_materials_depth3", ("json", None), 64, 48, {"samples": 4, "max_depth": 3}),
    ("all_materials_odd_size_spp", ("json", None), 37, 29, {"samples": 3}),
    ("all_materials_depth0", ("json", None), 20, 10, {"samples": 2, "max_depth": 0}),
]


def load_case(rtgo, loader):
    kind, name = loader
    if kind == "file":
        return rtgo.Scene.load_from_file(scene_path(name))
    return rtgo.Scene.from_json_text(all_materials_json())


def make_settings(rtgo, overrides, seed=1):
    st = rtgo.default_settings()
    st.seed = seed
    for k, v in overrides.items():
        setattr(st, k, v)
    return st


# Committed oracle fixtures (tests/golden/make_golden.py): (id, loader, w, h, overrides, seed)
GOLDEN_CASES = [
    ("spheres_facing", ("file", "sphere_reflections_light_facing.json"), 64, 48, {"samples": 4}, 1),
    ("silver_facing", ("file", "final_silver_prism_purple_cube_facing.json"), 64, 48, {"samples": 3}, 1),
    ("all_materials", ("json", None), 48, 32, {"samples": 4}, 7),
    ("all_materials_hard_depth4", ("json", None), 40, 24, {"samples": 2, "soft_shadows": 0, "max_depth": 4}, 2),
]


def spheres10k_scene(rtgo, n=10000):
    """The procedural C4/C5 scene (scenes/gen_spheres.py, SHA-256 pinned)."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("gen_spheres", scene_path("gen_spheres.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    return rtgo.Scene.from_json_text(g.dumps(g.generate(n)))


def _edge_scenes():
    """Scenes at the edges of the kernel's exact culling (rt_kernel.hip
    in_cone / cone_candidates, rt_schedule.hip pixel cones): their margins
    are relative (1e-7 .. 1e-5), so these stress huge radii, far
    coordinates, tiny spheres and a light almost on a surface."""
    def sph(p, r, m):
        return {"type": "sphere", "position": list(p), "radius": r, "material": m}

    metal = {"type": "metal", "color": [0.9, 0.8, 0.7], "roughness": 0.1}
    mirror = {"type": "metal", "color": [0.95, 0.95, 0.95], "roughness": 0.0, "metallic": 1.0}
    glass = {"type": "glass", "color": [0.95, 0.95, 1.0], "refractionIndex": 1.5}
    lamb = {"type": "lambertian", "color": [0.6, 0.5, 0.4]}
    out = {}
    # a radius-1e6 ground sphere (self-exclusion and cone tests at huge radius)
    out["huge_ground"] = {
        "camera": {"position": [0, 0.5, 6], "aspectRatio": 1.5},
        "objects": [sph((0, -1e6 - 1, 0), 1e6, lamb), sph((-1.5, 0, 0), 1, metal), sph((1.2, -0.2, 0.5), 0.8, glass),
                    sph((0, 0.4, -2), 1.4, mirror),
                    {"type": "cube", "position": [2.6, -0.5, 1.0], "size": [1, 1, 1], "material": metal}],
        "lights": [{"position": [5, 8, 6], "color": [1, 1, 1], "intensity": 80},
                   {"position": [-4, 2, 3], "color": [1, 0.8, 0.7], "intensity": 30}],
    }
    # the same scene around (1e5, 1e5, 1e5): camera, objects and lights
    off = (1e5, 1e5, 1e5)

    def shift(sc):
        sc = json.loads(json.dumps(sc))
        sc["camera"]["position"] = [a + b for a, b in zip(sc["camera"]["position"], off)]
        for o in sc["objects"]:
            o["position"] = [a + b for a, b in zip(o["position"], off)]
        for li in sc["lights"]:
            li["position"] = [a + b for a, b in zip(li["position"], off)]
        return sc

    far = shift(out["huge_ground"])
    far["objects"][0]["radius"] = 1e3  # (a 1e6 ground at 1e5 would swallow the camera)
    far["objects"][0]["position"][1] = off[1] - 1e3 - 1
    out["far_coordinates"] = far
    # radius-1e-3 spheres seen from 2 cm (culling margins of tiny bounding spheres)
    tiny = []
    for i in range(40):
        x = ((i * 37) % 13 - 6) * 2.3e-3
        y = ((i * 11) % 9 - 4) * 2.1e-3
        z = -0.02 - (i % 5) * 1.7e-3
        tiny.append(sph((x, y, z), 1e-3, [metal, glass, lamb, mirror][i % 4]))
    tiny.append(sph((0, -1e3 - 0.02, 0), 1e3, lamb))
    out["tiny_spheres"] = {
        "camera": {"position": [0, 0, 0], "aspectRatio": 1.5},
        "objects": tiny,
        "lights": [{"position": [0.01, 0.02, -0.01], "color": [1, 1, 1], "intensity": 0.002},
                   {"position": [-0.02, 0.01, 0.0], "color": [1, 0.9, 0.8], "intensity": 0.001}],
    }
    # lights 2e-3 and 5e-4 (< 0.001: skipped by renderer.go:252-254) above surfaces
    out["light_on_surface"] = {
        "camera": {"position": [0, 0.5, 6], "aspectRatio": 1.5},
        "objects": [sph((0, -1001, 0), 1000, lamb), sph((0, 0, 0), 1, metal), sph((2.2, 0, 0), 0.9, glass),
                    sph((-2.2, 0, 0), 0.9, lamb)],
        "lights": [{"position": [0, 1.002, 0], "color": [1, 1, 1], "intensity": 2},
                   {"position": [2.2, 0.9005, 0], "color": [1, 1, 1], "intensity": 2},
                   {"position": [-2.2, -0.1, 0.902], "color": [1, 0.7, 0.6], "intensity": 3},
                   {"position": [0, -0.998, 3], "color": [0.5, 0.5, 1], "intensity": 5}],
    }
    return out


EDGE_SCENES = _edge_scenes()


def _cube_scenes():
    """Rays inside cubes.  createCube (scene.go:150-190) winds every
    triangle so that its normal (triangle.go:29-33) points INTO the box:
    FrontFace (triangle.go:70-73) is true only for a hit from inside.  These
    scenes put hit points on the inner faces of glass / dielectric cubes, the
    camera inside a cube, lights inside and outside cubes, and cubes with
    negative sizes (mirrored: their normals point out), so every shadow-ray
    shortcut of the kernels (rt_kernel.hip cone_candidates: the hit object's
    self-exclusion; box slab pruning; quiet lights; primary-ray masks) meets
    both orientations."""
    def sph(p, r, m):
        return {"type": "sphere", "position": list(p), "radius": r, "material": m}

    def cube(p, s, m):
        return {"type": "cube", "position": list(p), "size": list(s), "material": m}

    glass = {"type": "glass", "color": [0.9, 0.95, 1.0], "refractionIndex": 1.5}
    diel = {"type": "dielectric", "refractionIndex": 1.33}
    lamb = {"type": "lambertian", "color": [0.7, 0.6, 0.5]}
    red = {"type": "lambertian", "color": [0.8, 0.2, 0.2]}
    metal = {"type": "metal", "color": [0.9, 0.8, 0.7], "roughness": 0.1, "metallic": 0.9}
    mirror = {"type": "metal", "color": [0.95, 0.95, 0.95], "roughness": 0.0, "metallic": 1.0}
    cam = {"position": [0, 0.5, 6], "aspectRatio": 1.5}
    out = {}
    # a glass and a dielectric cube in front of the camera, lights above and
    # behind them: refracted paths hit the inner faces, whose shadow rays
    # toward the lights must cross the cube's far faces
    out["glass_dielectric_cubes"] = {
        "camera": cam,
        "objects": [sph((0, -1001, 0), 1000, lamb), cube((-1.3, 0, 0), (1.6, 1.6, 1.6), glass),
                    cube((1.3, 0.1, 0.3), (1.4, 1.2, 1.4), diel), sph((0, 0.3, -2.5), 1.0, metal),
                    cube((0.2, -0.7, 2.0), (0.5, 0.5, 0.5), red)],
        "lights": [{"position": [0, 6, 1], "color": [1, 1, 1], "intensity": 60},
                   {"position": [-4, 1, -4], "color": [1, 0.9, 0.8], "intensity": 40}],
    }
    # the camera inside a large lambertian cube (every camera ray starts
    # inside it), a light inside it and one outside
    out["camera_inside_cube"] = {
        "camera": {"position": [0, 0, 2], "aspectRatio": 1.5},
        "objects": [cube((0, 0, 0), (10, 8, 10), lamb), sph((-1.2, -1.5, -2), 1.0, metal),
                    cube((1.5, 0.5, -2.5), (1.2, 1.2, 1.2), glass), sph((0.3, 1.6, -1.5), 0.6, diel)],
        "lights": [{"position": [1, 2.5, 0], "color": [1, 1, 1], "intensity": 20},
                   {"position": [0, 30, 0], "color": [1, 1, 1], "intensity": 900}],
    }
    # a light inside a glass cube, a second light outside
    out["light_inside_glass_cube"] = {
        "camera": cam,
        "objects": [sph((0, -1001, 0), 1000, lamb), cube((0, 0, 0), (2, 2, 2), glass),
                    sph((-2.3, -0.2, 0.5), 0.8, red), sph((2.3, 0, -0.5), 0.9, metal)],
        "lights": [{"position": [0, 0.2, 0], "color": [1, 1, 1], "intensity": 6},
                   {"position": [3, 7, 4], "color": [1, 1, 1], "intensity": 70}],
    }
    # negative sizes: one or three negative components mirror the box (its
    # normals then point out, so FrontFace means "from outside"), two restore
    # the inward winding; glass so that paths reach both sides
    out["mirrored_cubes"] = {
        "camera": cam,
        "objects": [sph((0, -1001, 0), 1000, lamb), cube((-2.2, 0, 0), (-1.4, 1.4, 1.4), glass),
                    cube((0, 0, 0.4), (-1.3, -1.3, 1.3), diel), cube((2.2, 0, 0), (-1.4, -1.4, -1.4), glass),
                    cube((0, 1.6, -1), (1.0, -0.6, 1.0), metal)],
        "lights": [{"position": [1, 6, 2], "color": [1, 1, 1], "intensity": 60},
                   {"position": [-3, 2, -5], "color": [0.8, 0.8, 1], "intensity": 40}],
    }
    # the camera inside a hollow mirror sphere around a glass cube and a light:
    # 50-bounce paths (the lone-path form, solo_path, runs them when built in)
    out["mirror_probe_glass_cube"] = {
        "camera": {"position": [0, 0, 3.2], "aspectRatio": 1.5},
        "objects": [sph((0, 0, 0), 5.0, mirror), cube((0, -0.2, 0), (1.6, 1.6, 1.6), glass),
                    sph((1.8, 1.2, -1.0), 0.5, lamb)],
        "lights": [{"position": [0, 3.2, 0.5], "color": [1, 1, 1], "intensity": 8},
                   {"position": [-2.5, -1.0, 1.5], "color": [1, 0.8, 0.6], "intensity": 5}],
    }
    # a glass cube and a lambertian cube among 70 spheres (more than 64: the
    # scene has no shadow-cone masks and scans linearly)
    field = [sph((0, -1001, 0), 1000, lamb)]
    for i in range(70):
        x = (i % 10) * 0.7 - 3.15
        z = -(i // 10) * 0.7 + 1.0
        field.append(sph((x, -0.8 + 0.1 * (i % 3), z), 0.22, [metal, glass, red, diel][i % 4]))
    field += [cube((-0.6, 0.2, 1.4), (1.0, 1.0, 1.0), glass), cube((1.1, 0.0, 0.6), (0.8, 0.8, 0.8), red)]
    out["cubes_among_70_spheres"] = {
        "camera": cam,
        "objects": field,
        "lights": [{"position": [0, 6, 3], "color": [1, 1, 1], "intensity": 60},
                   {"position": [-4, 2, -2], "color": [1, 0.9, 0.8], "intensity": 30}],
    }
    return out


CUBE_SCENES = _cube_scenes()
