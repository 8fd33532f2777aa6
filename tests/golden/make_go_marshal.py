#!/usr/bin/env python3
"""tests/golden/go_marshal_all_materials.json: the all-materials parity
scene (tests/scene_cases.py ALL_MATERIALS) as Go's json.Marshal writes a
*scene.Scene (internal/scene/scene.go:12-39): struct fields in declaration
order with their json tags, `size` always present (omitempty never omits a
struct), `radius` omitted when 0, Vec3 as [x, y, z] (Vec3.MarshalJSON,
internal/math/vector.go:195-197), map keys sorted, float64 in Go's shortest
form ('e' notation below 1e-6 or from 1e21, exponent without leading zero).
This is the byte stream the cgo shim (go/internal/renderer/gpu.go) hands to
rt_scene_parse_json.  Regenerate: python tests/golden/make_go_marshal.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from scene_cases import ALL_MATERIALS  # noqa: E402


def go_float(f):
    f = float(f)
    a = abs(f)
    if a != 0 and (a < 1e-6 or a >= 1e21):
        s = "%r" % f
        mant, exp = s.split("e")
        sign = exp[0] if exp[0] in "+-" else "+"
        digits = exp.lstrip("+-").lstrip("0") or "0"
        if len(digits) < 2 and sign == "+":
            digits = digits.rjust(2, "0")
        return f"{mant}e{sign}{digits}" if sign == "-" else f"{mant}e+{digits}"
    if a >= 1e16:  # Go's 'f' form up to 1e21 (Python's repr switches to 'e' at 1e16)
        return format(f, "f").rstrip("0").rstrip(".")
    s = repr(f)
    return s[:-2] if s.endswith(".0") else s


def enc(v):
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, float)):
        return go_float(v)
    if isinstance(v, str):
        return json.dumps(v)
    if isinstance(v, list):
        return "[" + ",".join(enc(x) for x in v) + "]"
    if isinstance(v, dict):  # a map[string]interface{}: sorted keys
        return "{" + ",".join(json.dumps(k) + ":" + enc(v[k]) for k in sorted(v)) + "}"
    raise TypeError(v)


def vec(v):
    return "[" + ",".join(go_float(x) for x in (v or (0, 0, 0))) + "]"


def struct(fields):
    return "{" + ",".join(json.dumps(k) + ":" + v for k, v in fields) + "}"


def marshal_scene(sc):
    c = sc["camera"]
    cam = struct([("position", vec(c.get("position"))), ("lookAt", vec(c.get("lookAt"))), ("up", vec(c.get("up"))),
                  ("fov", go_float(c.get("fov", 0))), ("aspectRatio", go_float(c.get("aspectRatio", 0)))])
    objs = []
    for o in sc["objects"]:
        f = [("type", json.dumps(o["type"])), ("position", vec(o.get("position"))), ("size", vec(o.get("size")))]
        if o.get("radius", 0):
            f.append(("radius", go_float(o["radius"])))
        f.append(("material", enc(o["material"])))
        objs.append(struct(f))
    lights = [struct([("type", json.dumps(l.get("type", ""))), ("position", vec(l.get("position"))),
                      ("color", vec(l.get("color"))), ("intensity", go_float(l.get("intensity", 0)))])
              for l in sc["lights"]]
    return struct([("camera", cam), ("objects", "[" + ",".join(objs) + "]"), ("lights", "[" + ",".join(lights) + "]")])


if __name__ == "__main__":
    path = os.path.join(HERE, "go_marshal_all_materials.json")
    with open(path, "w") as f:
        f.write(marshal_scene(ALL_MATERIALS))
    print(path)
