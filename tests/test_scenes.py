"""The procedural 10k-sphere scene of configs C4/C5 (BASELINE.json
configs[3..4]; scenes/gen_spheres.py): deterministic, pinned by SHA-256, and
loadable through the scene loader (scene.go:45-148 mirror)."""
import collections
import importlib.util
import json
import os

import rtgo
from conftest import ROOT


def _gen():
    spec = importlib.util.spec_from_file_location("gen_spheres", os.path.join(ROOT, "scenes", "gen_spheres.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_generator_is_pinned():
    g = _gen()
    text = g.dumps(g.generate(10000))
    assert g.sha256(text) == g.EXPECTED_SHA256[10000]
    assert g.dumps(g.generate(10000)) == text  # deterministic


def test_generator_follows_its_spec():
    g = _gen()
    sc = g.generate(2000)
    kinds = collections.Counter(o["material"]["type"] for o in sc["objects"])
    assert set(kinds) == {"metal", "glass", "lambertian"}
    # selector < 0.4 metal, < 0.7 glass, else lambertian
    assert abs(kinds["metal"] / 2000 - 0.4) < 0.05 and abs(kinds["glass"] / 2000 - 0.3) < 0.05
    for o in sc["objects"]:
        x, y, z = o["position"]
        assert -30 <= x <= 30 and -20 <= y <= 20 and -80 <= z <= -10 and 0.3 <= o["radius"] <= 1.0


def test_ten_thousand_spheres_load(tmp_path):
    g = _gen()
    p = tmp_path / "spheres10000.json"
    p.write_text(g.dumps(g.generate(10000)))
    s = rtgo.Scene.load_from_file(str(p))
    v = s.view
    assert v.num_objects == 10000 and v.num_lights == 2
    assert json.loads(p.read_text())["camera"]["aspectRatio"] == 1.78


def test_edge_scenes_are_not_black():
    """The culling edge scenes (GPU parity) actually show their objects."""
    import json

    import numpy as np

    import oracle
    import rtgo
    from scene_cases import EDGE_SCENES, make_settings

    for name, sc in EDGE_SCENES.items():
        scene = rtgo.Scene.from_json_text(json.dumps(sc))
        lin, rgba, _ = oracle.render(scene, 36, 24, make_settings(rtgo, {"samples": 1, "max_depth": 8}))
        assert np.mean(rgba[..., :3] > 0) > 0.2, name
