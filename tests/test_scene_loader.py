"""Scene JSON loader of librtgo (host code, CPU): the reference's
scene.LoadFromFile / CreateHittables behaviour (internal/scene/scene.go:12-224,
Vec3.UnmarshalJSON internal/math/vector.go:176-193)."""
import json
import os

import pytest

import rtgo
from conftest import SCENES


def load(obj):
    return rtgo.Scene.from_json_text(json.dumps(obj) if not isinstance(obj, str) else obj)


def objects(scene):
    return [scene.view.objects[i] for i in range(scene.num_objects)]


def test_committed_scenes_load():
    s = rtgo.Scene.load_from_file(os.path.join(SCENES, "sphere_reflections_light.json"))
    assert s.num_objects == 5 and s.view.num_lights == 2
    # object 2's metal material has no "color": Go panics (scene.go:113); we
    # default to the zero Vec3 and count a warning
    assert s.warnings == 1
    s = rtgo.Scene.load_from_file(os.path.join(SCENES, "final_silver_prism_purple_cube_.json"))
    assert s.num_objects == 2 and s.view.num_lights == 3  # triangularPrism: "Unknown object type", skipped


def test_facing_variants_change_only_the_camera():
    for name, z in (("sphere_reflections_light", 8.0), ("final_silver_prism_purple_cube_", 25.0)):
        a = json.load(open(os.path.join(SCENES, name + ".json")))
        b = json.load(open(os.path.join(SCENES, name.rstrip("_") + "_facing.json")))
        assert b["camera"]["position"][2] == z
        b["camera"]["position"][2] = a["camera"]["position"][2]
        assert a == b


def test_keys_are_case_insensitive_and_vec3_accepts_objects():
    s = load({
        "Camera": {"POSITION": {"x": 1, "y": 2, "z": 3}, "aspectratio": 1.25},
        "Objects": [{"Type": "sphere", "Position": [0, 0, -1], "RADIUS": 0.5,
                     "Material": {"type": "lambertian", "color": [0.1, 0.2, 0.3]}}],
        "LIGHTS": [{"Position": [1, 1, 1], "Color": [1, 1, 1], "Intensity": 2}],
    })
    cam = s.view.camera
    assert list(cam.position) == [1, 2, 3] and cam.aspect_ratio == 1.25
    (o,) = objects(s)
    assert o.type == rtgo.RT_OBJ_SPHERE and list(o.position) == [0, 0, -1] and o.radius == 0.5
    assert list(o.material.color) == [0.1, 0.2, 0.3]
    assert s.view.lights[0].intensity == 2


def test_material_defaults():  # scene.go:104-148, material.go:65-73
    mats = [{"type": "metal", "color": [1, 1, 1]},
            {"type": "shiny", "color": [1, 1, 1]},
            {"type": "glass", "color": [1, 1, 1]},
            {"type": "dielectric"},
            {"type": "perfectmirror", "color": [1, 1, 1]},
            {"type": "diffuselight", "color": [2, 2, 2]},
            {"type": "no-such-kind", "color": [0.5, 0.5, 0.5]}]
    s = load({"objects": [{"type": "sphere", "radius": 1, "material": m} for m in mats]})
    o = objects(s)
    K = rtgo.MATERIAL_KINDS
    assert o[0].material.kind == K["metal"] and o[0].material.roughness == 0.0
    assert o[0].material.metallic == 1.0 and o[0].material.specular == 1.0
    assert o[1].material.kind == K["shiny"] and o[1].material.metallic == 0.0
    assert o[2].material.refraction_index == 1.5 and o[3].material.refraction_index == 1.5
    assert o[4].material.kind == K["perfectmirror"]
    assert o[5].material.kind == K["diffuselight"]
    assert o[6].material.kind == K["lambertian"]  # unknown type -> default case


def test_unknown_object_types_are_skipped_and_printed(capfd):
    s = load({"objects": [
        {"type": "cube", "position": [0, 0, -5], "size": [1, 2, 3], "material": {"type": "metal", "color": [1, 1, 1]}},
        {"type": "triangularPrism", "material": {"type": "metal", "color": [1, 1, 1]}},
        {"type": "sphere", "position": [0, 0, -3], "radius": 0.5, "material": {"type": "glass", "color": [1, 1, 1]}},
    ]})
    assert [o.type for o in objects(s)] == [rtgo.RT_OBJ_CUBE, rtgo.RT_OBJ_SPHERE]
    s.print_hittables()
    out = capfd.readouterr().out
    # CreateHittables' stdout lines (scene.go:62-88)
    assert "Creating hittables from 3 scene objects..." in out
    assert "Created cube at {0 0 -5} with size {1 2 3}" in out
    assert "Unknown object type: triangularPrism" in out
    assert "Created 2 hittables total" in out


@pytest.mark.parametrize("text,fragment", [
    ("{bad json", "error parsing JSON"),
    ('{"objects": [{"type": "sphere", "material": {"type": "metal", "color": "red"}}]}', "color"),
    ('{"camera": 5}', "camera"),
    # material colours are read from a map as []interface{} (scene.go:211-217): no object form
    ('{"objects": [{"type": "sphere", "material": {"type": "glass", "color": {"x": 1, "y": 1, "z": 1}}}]}', "color"),
    ('{"objects": {}}', "objects"),
    ("[1, 2] x", "error parsing JSON"),
])
def test_parse_errors_are_reported_not_fatal(text, fragment):
    with pytest.raises(rtgo.RenderError) as e:
        load(text)
    assert fragment in str(e.value)


def test_missing_file_is_an_error():
    with pytest.raises(rtgo.RenderError):
        rtgo.Scene.load_from_file(os.path.join(SCENES, "does-not-exist.json"))


def test_from_python_matches_json_loader():
    obj = json.load(open(os.path.join(SCENES, "sphere_reflections_light_facing.json")))
    a = rtgo.Scene.load_from_file(os.path.join(SCENES, "sphere_reflections_light_facing.json"))
    b = rtgo.Scene.from_python(obj["camera"], obj["objects"], obj["lights"])
    assert a.num_objects == b.num_objects
    for x, y in zip(objects(a), objects(b)):
        assert bytes(x) == bytes(y)
