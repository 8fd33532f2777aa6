// scene_json.cpp — the reference's JSON scene surface.
//
// Mirrors scene.LoadFromFile (internal/scene/scene.go:45-57: os.ReadFile +
// encoding/json into Scene), Vec3.UnmarshalJSON (internal/math/vector.go:
// 176-193: [x,y,z] or {"X":..,"Y":..,"Z":..}), and the material decoding of
// createMaterial (scene.go:104-148) including its defaults.  encoding/json
// rules kept: object keys match struct fields case-insensitively, the last
// duplicate wins, unknown keys are ignored, a type mismatch is an error.
// Where Go panics at render time (a material without "type", a missing or
// malformed "color" array, a non-number parameter: scene.go:105-145,
// 211-224) this loader returns RT_E_PARSE — except a missing "color", which
// is loaded as (0,0,0) with a warning so that the benchmark scene
// demo-assets/sphere_reflections_light.json (object 2 has no color) loads
// (SURVEY.md §8d).
#include <errno.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "rt_internal.h"

namespace rtgo {

// ------------------------------------------------------------ JSON value
struct JVal {
  enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
  bool b = false;
  double num = 0;
  std::string str;
  std::vector<JVal> arr;
  std::vector<std::pair<std::string, JVal>> obj;  // in document order
};

struct JParser {
  const char* p;
  const char* end;
  std::string err;
  int depth = 0;

  void ws() {
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  bool fail(const std::string& m) {
    if (err.empty()) err = m;
    return false;
  }
  bool lit(const char* s) {
    size_t n = strlen(s);
    if ((size_t)(end - p) < n || memcmp(p, s, n) != 0) return false;
    p += n;
    return true;
  }
  static void utf8(std::string& out, unsigned cp) {
    if (cp < 0x80) {
      out += (char)cp;
    } else if (cp < 0x800) {
      out += (char)(0xC0 | (cp >> 6));
      out += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18));
      out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    }
  }
  bool hex4(unsigned& v) {
    if (end - p < 4) return false;
    v = 0;
    for (int i = 0; i < 4; ++i) {
      char ch = p[i];
      v <<= 4;
      if (ch >= '0' && ch <= '9') v |= ch - '0';
      else if (ch >= 'a' && ch <= 'f') v |= ch - 'a' + 10;
      else if (ch >= 'A' && ch <= 'F') v |= ch - 'A' + 10;
      else return false;
    }
    p += 4;
    return true;
  }
  bool string(std::string& out) {
    if (p >= end || *p != '"') return fail("expected string");
    ++p;
    while (p < end && *p != '"') {
      unsigned char ch = (unsigned char)*p;
      if (ch < 0x20) return fail("invalid character in string literal");
      if (ch == '\\') {
        ++p;
        if (p >= end) return fail("unexpected end of JSON input");
        char e = *p++;
        switch (e) {
          case '"': out += '"'; break;
          case '\\': out += '\\'; break;
          case '/': out += '/'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'n': out += '\n'; break;
          case 'r': out += '\r'; break;
          case 't': out += '\t'; break;
          case 'u': {
            unsigned cp;
            if (!hex4(cp)) return fail("invalid \\u escape");
            if (cp >= 0xD800 && cp < 0xDC00 && end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
              const char* save = p;
              p += 2;
              unsigned lo;
              if (hex4(lo) && lo >= 0xDC00 && lo < 0xE000) {
                cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
              } else {
                p = save;
                cp = 0xFFFD;
              }
            } else if (cp >= 0xD800 && cp < 0xE000) {
              cp = 0xFFFD;
            }
            utf8(out, cp);
            break;
          }
          default: return fail("invalid escape in string literal");
        }
      } else {
        out += (char)ch;
        ++p;
      }
    }
    if (p >= end) return fail("unexpected end of JSON input");
    ++p;
    return true;
  }
  bool number(double& v) {
    const char* s = p;
    if (p < end && *p == '-') ++p;
    if (p >= end) return fail("unexpected end of JSON input");
    if (*p == '0') {
      ++p;
    } else if (*p >= '1' && *p <= '9') {
      while (p < end && *p >= '0' && *p <= '9') ++p;
    } else {
      return fail("invalid character in numeric literal");
    }
    if (p < end && *p == '.') {
      ++p;
      if (p >= end || !(*p >= '0' && *p <= '9')) return fail("invalid character after decimal point");
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    if (p < end && (*p == 'e' || *p == 'E')) {
      ++p;
      if (p < end && (*p == '+' || *p == '-')) ++p;
      if (p >= end || !(*p >= '0' && *p <= '9')) return fail("invalid character in exponent");
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    std::string tok(s, p);
    errno = 0;
    v = strtod(tok.c_str(), nullptr);  // correctly rounded, like strconv.ParseFloat
    if (errno == ERANGE && (isinf(v))) return fail("number " + tok + " out of range");
    return true;
  }
  bool value(JVal& v) {
    if (++depth > 10000) return fail("exceeded max depth");
    ws();
    if (p >= end) return fail("unexpected end of JSON input");
    bool ok = true;
    if (*p == '{') {
      ++p;
      v.kind = JVal::OBJ;
      ws();
      if (p < end && *p == '}') {
        ++p;
      } else {
        for (;;) {
          ws();
          std::string k;
          if (!string(k)) return false;
          ws();
          if (p >= end || *p != ':') return fail("expected ':' after object key");
          ++p;
          JVal child;
          if (!value(child)) return false;
          v.obj.emplace_back(std::move(k), std::move(child));
          ws();
          if (p < end && *p == ',') {
            ++p;
            continue;
          }
          if (p < end && *p == '}') {
            ++p;
            break;
          }
          return fail("expected ',' or '}' after object value");
        }
      }
    } else if (*p == '[') {
      ++p;
      v.kind = JVal::ARR;
      ws();
      if (p < end && *p == ']') {
        ++p;
      } else {
        for (;;) {
          JVal child;
          if (!value(child)) return false;
          v.arr.push_back(std::move(child));
          ws();
          if (p < end && *p == ',') {
            ++p;
            continue;
          }
          if (p < end && *p == ']') {
            ++p;
            break;
          }
          return fail("expected ',' or ']' after array element");
        }
      }
    } else if (*p == '"') {
      v.kind = JVal::STR;
      ok = string(v.str);
    } else if (*p == 't') {
      if (!lit("true")) return fail("invalid literal");
      v.kind = JVal::BOOL;
      v.b = true;
    } else if (*p == 'f') {
      if (!lit("false")) return fail("invalid literal");
      v.kind = JVal::BOOL;
    } else if (*p == 'n') {
      if (!lit("null")) return fail("invalid literal");
      v.kind = JVal::NUL;
    } else {
      v.kind = JVal::NUM;
      ok = number(v.num);
    }
    --depth;
    return ok;
  }
};

// Go's case-insensitive field match (encoding/json uses EqualFold; the
// scene's field names are ASCII).
static bool key_is(const std::string& k, const char* name) { return strcasecmp(k.c_str(), name) == 0; }

struct LoadCtx {
  std::string err;
  int warnings = 0;
  bool fail(const std::string& m) {
    if (err.empty()) err = m;
    return false;
  }
};

// Vec3.UnmarshalJSON (vector.go:176-193)
static bool get_vec3(const JVal& v, double out[3], LoadCtx& L, const std::string& what) {
  if (v.kind == JVal::ARR) {
    for (const JVal& e : v.arr)
      if (e.kind != JVal::NUM) return L.fail(what + ": Vec3 array element is not a number");
    if (v.arr.size() != 3)
      return L.fail(what + ": expected 3 elements for Vec3, got " + std::to_string(v.arr.size()));
    for (int i = 0; i < 3; ++i) out[i] = v.arr[i].num;
    return true;
  }
  if (v.kind == JVal::NUL) return L.fail(what + ": expected 3 elements for Vec3, got 0");
  if (v.kind != JVal::OBJ) return L.fail(what + ": cannot unmarshal into Vec3");
  double r[3] = {0, 0, 0};
  for (const auto& kv : v.obj) {
    int idx = key_is(kv.first, "X") ? 0 : key_is(kv.first, "Y") ? 1 : key_is(kv.first, "Z") ? 2 : -1;
    if (idx < 0) continue;
    if (kv.second.kind == JVal::NUL) continue;
    if (kv.second.kind != JVal::NUM) return L.fail(what + ": Vec3 field is not a number");
    r[idx] = kv.second.num;
  }
  for (int i = 0; i < 3; ++i) out[i] = r[i];
  return true;
}

static bool get_num(const JVal& v, double& out, LoadCtx& L, const std::string& what) {
  if (v.kind == JVal::NUL) return true;  // null leaves a Go float64 unchanged
  if (v.kind != JVal::NUM) return L.fail("cannot unmarshal into Go struct field " + what + " of type float64");
  out = v.num;
  return true;
}

static bool get_str(const JVal& v, std::string& out, LoadCtx& L, const std::string& what) {
  if (v.kind == JVal::NUL) return true;
  if (v.kind != JVal::STR) return L.fail("cannot unmarshal into Go struct field " + what + " of type string");
  out = v.str;
  return true;
}

// Material map (scene.go:31) as the Go %v printer and createMaterial see it.
struct RawMat {
  bool present = false;   // "material" key present and an object
  bool is_null = false;
  std::map<std::string, const JVal*> m;  // exact keys (map[string]interface{} is case-sensitive)
};

// A scene object as parsed (before the unknown-type filter).
struct RawObject {
  std::string type;
  double position[3] = {0, 0, 0};
  double size[3] = {0, 0, 0};
  double radius = 0;
  std::string mat_type_repr;  // fmt %s of obj.Material["type"]
  bool known = false;
};

static std::string go_s_repr(const JVal* v) {
  if (!v || v->kind == JVal::NUL) return "%!s(<nil>)";
  switch (v->kind) {
    case JVal::STR: return v->str;
    case JVal::BOOL: return v->b ? "%!s(bool=true)" : "%!s(bool=false)";
    case JVal::NUM: {
      char b[64];
      snprintf(b, sizeof b, "%%!s(float64=%.17g)", v->num);
      return b;
    }
    case JVal::ARR: return "[...]";
    default: return "map[...]";
  }
}

// createMaterial, scene.go:104-148 — the loader's defaults.
static bool decode_material(const RawMat& rm, rt_material& out, LoadCtx& L, int obj_index) {
  const std::string where = "object " + std::to_string(obj_index + 1) + " material";
  memset(&out, 0, sizeof out);
  if (!rm.present) return L.fail(where + ": missing (Go panics: nil map has no \"type\", scene.go:105)");
  auto it = rm.m.find("type");
  if (it == rm.m.end() || it->second->kind != JVal::STR)
    return L.fail(where + ": \"type\" is not a string (Go panics, scene.go:105)");
  const std::string& t = it->second->str;
  auto color = [&](bool required) -> bool {
    auto c = rm.m.find("color");
    if (c == rm.m.end() || c->second->kind == JVal::NUL) {
      if (!required) return true;
      ++L.warnings;
      fprintf(stderr,
              "warning: %s: \"%s\" material has no \"color\"; using (0,0,0) (the Go loader panics here, "
              "internal/scene/scene.go:113)\n",
              where.c_str(), t.c_str());
      return true;
    }
    const JVal& a = *c->second;
    if (a.kind != JVal::ARR || a.arr.size() < 3)
      return L.fail(where + ": \"color\" must be an array of at least 3 numbers (Go panics, scene.go:211-217)");
    for (int i = 0; i < 3; ++i) {
      if (a.arr[i].kind != JVal::NUM) return L.fail(where + ": \"color\" element is not a number");
      out.color[i] = a.arr[i].num;
    }
    return true;
  };
  auto num = [&](const char* key, double def, double& dst) -> bool {
    auto c = rm.m.find(key);
    dst = def;
    if (c == rm.m.end()) return true;
    if (c->second->kind != JVal::NUM)
      return L.fail(where + ": \"" + key + "\" is not a number (Go panics, scene.go:221)");
    dst = c->second->num;
    return true;
  };
  if (t == "lambertian") {
    out.kind = RT_MAT_LAMBERTIAN;
    return color(true);
  } else if (t == "metal") {
    out.kind = RT_MAT_METAL;
    return color(true) && num("roughness", 0.0, out.roughness) && num("metallic", 1.0, out.metallic) &&
           num("specular", 1.0, out.specular);
  } else if (t == "shiny") {
    out.kind = RT_MAT_SHINY;
    return color(true) && num("roughness", 0.0, out.roughness) && num("metallic", 0.0, out.metallic) &&
           num("specular", 1.0, out.specular);
  } else if (t == "perfectmirror") {
    out.kind = RT_MAT_PERFECTMIRROR;
    return color(true) && num("roughness", 0.0, out.roughness);
  } else if (t == "glass") {
    out.kind = RT_MAT_GLASS;
    return color(true) && num("refractionIndex", 1.5, out.refraction_index);
  } else if (t == "dielectric") {
    out.kind = RT_MAT_DIELECTRIC;
    return num("refractionIndex", 1.5, out.refraction_index);
  } else if (t == "diffuselight") {
    out.kind = RT_MAT_DIFFUSELIGHT;
    return color(true);
  }
  out.kind = RT_MAT_LAMBERTIAN;  // default case
  return color(true);
}

}  // namespace rtgo

using namespace rtgo;

struct rt_scene_buf {
  rt_scene view;
  std::vector<rt_object> objects;
  std::vector<rt_light> lights;
  std::vector<RawObject> raw;  // every JSON object, for the reference's stdout lines
  int warnings = 0;
};

namespace rtgo {

static bool load_scene(const JVal& root, rt_scene_buf& sb, LoadCtx& L) {
  if (root.kind == JVal::NUL) return true;  // json "null" into a struct: no-op
  if (root.kind != JVal::OBJ) return L.fail("cannot unmarshal non-object into Go value of type scene.Scene");
  rt_camera& cam = sb.view.camera;
  memset(&cam, 0, sizeof cam);
  // JSON objects and lights are decoded into fresh slices (last duplicate key wins)
  const JVal* objs = nullptr;
  const JVal* lights = nullptr;
  bool have_objs = false, have_lights = false;
  for (const auto& kv : root.obj) {
    if (key_is(kv.first, "camera")) {
      const JVal& c = kv.second;
      if (c.kind == JVal::NUL) continue;
      if (c.kind != JVal::OBJ) return L.fail("cannot unmarshal into Go struct field Scene.camera");
      for (const auto& ck : c.obj) {
        if (key_is(ck.first, "position")) {
          if (!get_vec3(ck.second, cam.position, L, "camera.position")) return false;
        } else if (key_is(ck.first, "lookAt")) {
          if (!get_vec3(ck.second, cam.look_at, L, "camera.lookAt")) return false;
        } else if (key_is(ck.first, "up")) {
          if (!get_vec3(ck.second, cam.up, L, "camera.up")) return false;
        } else if (key_is(ck.first, "fov")) {
          if (!get_num(ck.second, cam.fov, L, "Camera.fov")) return false;
        } else if (key_is(ck.first, "aspectRatio")) {
          if (!get_num(ck.second, cam.aspect_ratio, L, "Camera.aspectRatio")) return false;
        }
      }
    } else if (key_is(kv.first, "objects")) {
      objs = &kv.second;
      have_objs = true;
    } else if (key_is(kv.first, "lights")) {
      lights = &kv.second;
      have_lights = true;
    }
  }
  if (have_objs && objs->kind != JVal::NUL) {
    if (objs->kind != JVal::ARR) return L.fail("cannot unmarshal into Go struct field Scene.objects");
    for (size_t i = 0; i < objs->arr.size(); ++i) {
      const JVal& o = objs->arr[i];
      RawObject ro;
      RawMat rm;
      if (o.kind == JVal::NUL) {
        // a null element decodes to a zero Object
      } else if (o.kind != JVal::OBJ) {
        return L.fail("cannot unmarshal into Go value of type scene.Object");
      } else {
        for (const auto& ok : o.obj) {
          const std::string w = "objects[" + std::to_string(i) + "]." + ok.first;
          if (key_is(ok.first, "type")) {
            if (!get_str(ok.second, ro.type, L, "Object.type")) return false;
          } else if (key_is(ok.first, "position")) {
            if (!get_vec3(ok.second, ro.position, L, w)) return false;
          } else if (key_is(ok.first, "size")) {
            if (!get_vec3(ok.second, ro.size, L, w)) return false;
          } else if (key_is(ok.first, "radius")) {
            if (!get_num(ok.second, ro.radius, L, "Object.radius")) return false;
          } else if (key_is(ok.first, "material")) {
            if (ok.second.kind == JVal::NUL) {
              rm = RawMat();
              rm.is_null = true;
            } else if (ok.second.kind != JVal::OBJ) {
              return L.fail("cannot unmarshal into Go struct field Object.material");
            } else {
              // decoding into an existing map merges keys
              rm.present = true;
              for (const auto& mk : ok.second.obj) rm.m[mk.first] = &mk.second;
            }
          }
        }
      }
      auto t = rm.m.find("type");
      ro.mat_type_repr = go_s_repr(t == rm.m.end() ? nullptr : t->second);
      ro.known = ro.type == "sphere" || ro.type == "cube";
      if (ro.known) {
        rt_object ob;
        memset(&ob, 0, sizeof ob);
        ob.type = ro.type == "sphere" ? RT_OBJ_SPHERE : RT_OBJ_CUBE;
        memcpy(ob.position, ro.position, sizeof ob.position);
        memcpy(ob.size, ro.size, sizeof ob.size);
        ob.radius = ro.radius;
        if (!decode_material(rm, ob.material, L, (int)i)) return false;
        sb.objects.push_back(ob);
      }
      sb.raw.push_back(ro);
    }
  }
  if (have_lights && lights->kind != JVal::NUL) {
    if (lights->kind != JVal::ARR) return L.fail("cannot unmarshal into Go struct field Scene.lights");
    for (size_t i = 0; i < lights->arr.size(); ++i) {
      const JVal& l = lights->arr[i];
      rt_light rl;
      memset(&rl, 0, sizeof rl);
      if (l.kind == JVal::OBJ) {
        for (const auto& lk : l.obj) {
          const std::string w = "lights[" + std::to_string(i) + "]." + lk.first;
          if (key_is(lk.first, "position")) {
            if (!get_vec3(lk.second, rl.position, L, w)) return false;
          } else if (key_is(lk.first, "color")) {
            if (!get_vec3(lk.second, rl.color, L, w)) return false;
          } else if (key_is(lk.first, "intensity")) {
            if (!get_num(lk.second, rl.intensity, L, "Light.intensity")) return false;
          } else if (key_is(lk.first, "type")) {
            std::string ignored;
            if (!get_str(lk.second, ignored, L, "Light.type")) return false;
          }
        }
      } else if (l.kind != JVal::NUL) {
        return L.fail("cannot unmarshal into Go value of type scene.Light");
      }
      sb.lights.push_back(rl);
    }
  }
  return true;
}

// Go's %v for a float64: strconv.FormatFloat(v, 'g', -1, 64) — the shortest
// round-tripping digits, in %e form when exp < -4 || exp >= 6 (strconv
// uses precision 6 for that decision when the precision is shortest).
std::string go_fmt_float(double v) {
  if (isnan(v)) return "NaN";
  if (isinf(v)) return v > 0 ? "+Inf" : "-Inf";
  if (v == 0) return signbit(v) ? "-0" : "0";
  char buf[64];
  int prec = 1;
  for (; prec <= 17; ++prec) {
    snprintf(buf, sizeof buf, "%.*e", prec - 1, v);
    if (strtod(buf, nullptr) == v) break;
  }
  // buf = [-]d.ddde[+-]xx ; extract digits and exponent
  std::string s(buf);
  bool neg = s[0] == '-';
  if (neg) s = s.substr(1);
  size_t epos = s.find('e');
  std::string mant = s.substr(0, epos);
  int exp10 = atoi(s.c_str() + epos + 1);
  std::string digits;
  for (char ch : mant)
    if (ch != '.') digits += ch;
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  std::string out;
  if (exp10 < -4 || exp10 >= 6) {
    out = digits.substr(0, 1);
    if (digits.size() > 1) out += "." + digits.substr(1);
    char eb[16];
    snprintf(eb, sizeof eb, "e%c%02d", exp10 < 0 ? '-' : '+', abs(exp10));
    out += eb;
  } else if (exp10 < 0) {
    out = "0." + std::string(-exp10 - 1, '0') + digits;
  } else if ((int)digits.size() <= exp10 + 1) {
    out = digits + std::string(exp10 + 1 - digits.size(), '0');
  } else {
    out = digits.substr(0, exp10 + 1) + "." + digits.substr(exp10 + 1);
  }
  return neg ? "-" + out : out;
}

static std::string go_vec(const double v[3]) {
  return "{" + go_fmt_float(v[0]) + " " + go_fmt_float(v[1]) + " " + go_fmt_float(v[2]) + "}";
}

}  // namespace rtgo

extern "C" {

int rt_scene_print_hittables(const rt_scene_buf* b);

int rt_scene_parse_json(const char* text, size_t len, int32_t verbose, rt_scene_buf** out) {
  if (!out || (!text && len)) {
    set_error("invalid arguments");
    return RT_E_INVALID;
  }
  *out = nullptr;
  JParser jp{text, text + len};
  JVal root;
  if (!jp.value(root)) {
    set_error("error parsing JSON: " + jp.err);
    return RT_E_PARSE;
  }
  jp.ws();
  if (jp.p != jp.end) {
    set_error("error parsing JSON: invalid character after top-level value");
    return RT_E_PARSE;
  }
  std::unique_ptr<rt_scene_buf> sb(new rt_scene_buf());
  memset(&sb->view, 0, sizeof sb->view);
  LoadCtx L;
  if (!load_scene(root, *sb, L)) {
    set_error("error parsing JSON: " + L.err);
    return RT_E_PARSE;
  }
  sb->warnings = L.warnings;
  sb->view.objects = sb->objects.data();
  sb->view.num_objects = (int32_t)sb->objects.size();
  sb->view.lights = sb->lights.data();
  sb->view.num_lights = (int32_t)sb->lights.size();
  // verbose: the lines GetHittables prints when Render flattens the scene
  // (scene.go:62-88); a cgo caller that parses inside its Render wants them
  // here (go/internal/renderer/gpu.go)
  if (verbose) rt_scene_print_hittables(sb.get());
  *out = sb.release();
  return RT_OK;
}

int rt_scene_load_json(const char* path, int32_t verbose, rt_scene_buf** out) {
  if (!path || !out) {
    set_error("invalid arguments");
    return RT_E_INVALID;
  }
  FILE* f = fopen(path, "rb");
  if (!f) {
    set_error(std::string("error reading file: open ") + path + ": " + strerror(errno));
    return RT_E_IO;
  }
  std::string data;
  char buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) data.append(buf, n);
  bool bad = ferror(f);
  fclose(f);
  if (bad) {
    set_error(std::string("error reading file: ") + path);
    return RT_E_IO;
  }
  return rt_scene_parse_json(data.data(), data.size(), verbose, out);
}

const rt_scene* rt_scene_view(const rt_scene_buf* b) { return b ? &b->view : nullptr; }
int32_t rt_scene_warnings(const rt_scene_buf* b) { return b ? b->warnings : 0; }
void rt_scene_free(rt_scene_buf* b) { delete b; }

// The lines GetHittables prints (scene.go:62-88), for the CLI.
int rt_scene_print_hittables(const rt_scene_buf* b) {
  if (!b) return RT_E_INVALID;
  printf("Creating hittables from %zu scene objects...\n", b->raw.size());
  int created = 0;
  for (size_t i = 0; i < b->raw.size(); ++i) {
    const RawObject& o = b->raw[i];
    printf("  Processing object %zu: Type=%s, Material=%s\n", i + 1, o.type.c_str(), o.mat_type_repr.c_str());
    if (o.type == "sphere") {
      printf("    Created sphere at %s with radius %.1f\n", go_vec(o.position).c_str(), o.radius);
      ++created;
    } else if (o.type == "cube") {
      printf("    Created cube at %s with size %s\n", go_vec(o.position).c_str(), go_vec(o.size).c_str());
      ++created;
    } else {
      printf("    Unknown object type: %s\n", o.type.c_str());
    }
  }
  printf("Created %d hittables total\n", created);
  fflush(stdout);  // interleave correctly with the caller's own stdout writes
  return RT_OK;
}

}  // extern "C"
