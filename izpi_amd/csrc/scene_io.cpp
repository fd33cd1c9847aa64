// scene_io.cpp — scene ingestion in C++: the inputs that reach
// the hot path from files, for hosts without the Go toolchain.
//
//   transport.Scene from .pbtxt   prototext.Unmarshal     internal/leader/leader.go:64-71
//   transport.Scene from .izpi    proto.Unmarshal          internal/leader/leader.go:56-63
//   (schema: internal/proto/transport/transport.proto:1-313)
//   transport.ToScene up to the BVH: materials, textures, light-source library, camera,
//   embedded + streamed triangles, spheres   internal/transport/transport.go:53-689
//   light-source library / NewBlackbodySPD   internal/lightsources/lightsources.go:6-480,
//                                            internal/spectral/spectral.go:275-318
//   Wavefront OBJ + MTL, Scale/Rotate/Translate, GroupToTransportTrianglesWithMaterial
//                                            internal/wavefront/wavefront.go:107-625
//
// The output is an izpi_scene_input (include/izpi_host.h) — the same struct the
// Python harness fills — so the BVH build, the kernels and the oracle see one format.
//
// One protobuf decoder serves both encodings: text and wire format are parsed into the
// same field tree, driven by one schema table, and one converter walks that tree.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <errno.h>
#include <ctype.h>
#include <math.h>

#include <algorithm>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/izpi_host.h"
#include "cie_tables.h"
#include "gomath.h"
#include "lightsources.h"

namespace izpi_internal {
void set_host_error(const std::string& s);
}

namespace {

using izpi_internal::set_host_error;

struct Fail {
  int code;
  std::string msg;
};
[[noreturn]] void fail(int code, const std::string& m) { throw Fail{code, m}; }
[[noreturn]] void invalid(const std::string& m) { fail(IZPI_ERR_INVALID, m); }

// ---------------------------------------------------------------- number parsing
// strconv.ParseFloat(s, 64|32): the whole string, no surrounding space; correctly
// rounded (strtod / strtof round directly from the decimal string, as Go does for
// bitSize 32). Out of range is an error; underflow to zero is not.
bool go_parse_float(const std::string& s, bool f32, double* out) {
  if (s.empty() || isspace((unsigned char)s[0])) return false;
  errno = 0;
  char* end = nullptr;
  double v;
  if (f32) {
    float f = strtof(s.c_str(), &end);
    v = (double)f;
  } else {
    v = strtod(s.c_str(), &end);
  }
  if (end != s.c_str() + s.size()) return false;
  if (errno == ERANGE && (v == HUGE_VAL || v == -HUGE_VAL)) return false;
  *out = v;
  return true;
}

// strconv.ParseInt(s, 10, 32)
bool go_parse_int32(const std::string& s, int64_t* out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
  if (i == s.size()) return false;
  int64_t v = 0;
  for (; i < s.size(); i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (s[i] - '0');
    if (v > (int64_t)1 << 32) return false;
  }
  v = neg ? -v : v;
  if (v < INT32_MIN || v > INT32_MAX) return false;
  *out = v;
  return true;
}

// strings.Split(s, " ")
std::vector<std::string> split_space(const std::string& s) {
  std::vector<std::string> out;
  size_t b = 0;
  for (;;) {
    size_t e = s.find(' ', b);
    if (e == std::string::npos) { out.push_back(s.substr(b)); break; }
    out.push_back(s.substr(b, e - b));
    b = e + 1;
  }
  return out;
}

bool has_prefix(const std::string& s, const char* p) { return s.compare(0, strlen(p), p) == 0; }

// bufio.Scanner line splitting: '\n' separated, one trailing '\r' dropped
std::vector<std::string> scan_lines(const char* text, uint64_t len) {
  std::vector<std::string> lines;
  uint64_t b = 0;
  while (b < len) {
    uint64_t e = b;
    while (e < len && text[e] != '\n') e++;
    uint64_t ee = e;
    if (ee > b && text[ee - 1] == '\r') ee--;
    lines.emplace_back(text + b, text + ee);
    b = e + 1;
  }
  return lines;
}

// ======================================================================= protobuf
enum FT { T_DOUBLE, T_FLOAT, T_UINT32, T_UINT64, T_BOOL, T_STRING, T_ENUM, T_MSG };

struct FieldDef {
  const char* name;
  int num;
  FT type;
  const char* sub;  // message or enum type
  bool repeated;
  int oneof;        // 0 = none, else a group id unique within the message
};

struct MsgDef {
  const char* name;
  std::vector<FieldDef> fields;
  int find(const std::string& n) const {
    for (size_t i = 0; i < fields.size(); i++)
      if (n == fields[i].name) return (int)i;
    return -1;
  }
  int find_num(int num) const {
    for (size_t i = 0; i < fields.size(); i++)
      if (fields[i].num == num) return (int)i;
    return -1;
  }
};

struct EnumDef {
  const char* name;
  std::vector<std::pair<const char*, int>> values;
};

// transport.proto:1-313 (the message types a Scene reaches)
const std::vector<EnumDef>& enums() {
  static const std::vector<EnumDef> e = {
      {"TextureType", {{"TEXTURE_TYPE_UNSPECIFIED", 0}, {"CONSTANT", 1}, {"CHECKER", 2}, {"IMAGE", 3}, {"NOISE", 4},
                       {"SPECTRAL_CONSTANT", 5}, {"SPECTRAL_CHECKER", 6}}},
      {"TexturePixelFormat", {{"TEXTURE_PIXEL_FORMAT_UNSPECIFIED", 0}, {"FLOAT64", 1}}},
      {"MaterialType", {{"MATERIAL_TYPE_UNSPECIFIED", 0}, {"DIELECTRIC", 1}, {"DIFFUSE_LIGHT", 2}, {"ISOTROPIC", 3},
                        {"LAMBERT", 4}, {"METAL", 5}, {"PBR", 6}}},
      {"ColourRepresentation", {{"COLOUR_REPRESENTATION_UNSPECIFIED", 0}, {"RGB", 1}, {"SPECTRAL", 2}}},
      {"GeometryOperator", {{"GEOMETRY_OPERATOR_UNSPECIFIED", 0}, {"DISPLACE", 1}}},
  };
  return e;
}

const std::vector<MsgDef>& messages() {
  static const std::vector<MsgDef> m = {
      {"Vec3", {{"x", 1, T_FLOAT, nullptr, false, 0}, {"y", 2, T_FLOAT, nullptr, false, 0}, {"z", 3, T_FLOAT, nullptr, false, 0}}},
      {"Vec2", {{"u", 1, T_FLOAT, nullptr, false, 0}, {"v", 2, T_FLOAT, nullptr, false, 0}}},
      {"Camera",
       {{"lookfrom", 1, T_MSG, "Vec3", false, 0}, {"lookat", 2, T_MSG, "Vec3", false, 0}, {"vup", 3, T_MSG, "Vec3", false, 0},
        {"vfov", 4, T_FLOAT, nullptr, false, 0}, {"aspect", 5, T_FLOAT, nullptr, false, 0},
        {"aperture", 6, T_FLOAT, nullptr, false, 0}, {"focusdist", 7, T_FLOAT, nullptr, false, 0},
        {"time0", 8, T_FLOAT, nullptr, false, 0}, {"time1", 9, T_FLOAT, nullptr, false, 0},
        {"exposure", 10, T_FLOAT, nullptr, false, 0}}},
      {"ImageTextureMetadata",
       {{"filename", 1, T_STRING, nullptr, false, 0}, {"width", 2, T_UINT32, nullptr, false, 0},
        {"height", 3, T_UINT32, nullptr, false, 0}, {"channels", 4, T_UINT32, nullptr, false, 0},
        {"pixel_format", 5, T_ENUM, "TexturePixelFormat", false, 0}}},
      {"DisplaceOperator",
       {{"min", 1, T_DOUBLE, nullptr, false, 0}, {"max", 2, T_DOUBLE, nullptr, false, 0},
        {"displacement_map", 3, T_STRING, nullptr, false, 0}}},
      {"Texture",
       {{"name", 1, T_STRING, nullptr, false, 0}, {"type", 2, T_ENUM, "TextureType", false, 0},
        {"constant", 3, T_MSG, "ConstantTexture", false, 1}, {"checker", 4, T_MSG, "CheckerTexture", false, 1},
        {"image", 5, T_MSG, "ImageTexture", false, 1}, {"noise", 6, T_MSG, "NoiseTexture", false, 1},
        {"spectral_constant", 7, T_MSG, "SpectralConstantTexture", false, 1},
        {"spectral_checker", 8, T_MSG, "SpectralCheckerTexture", false, 1}}},
      {"ConstantTexture", {{"value", 1, T_MSG, "Vec3", false, 0}}},
      {"CheckerTexture", {{"odd", 1, T_MSG, "Texture", false, 0}, {"even", 2, T_MSG, "Texture", false, 0}}},
      {"ImageTexture", {{"filename", 1, T_STRING, nullptr, false, 0}}},
      {"NoiseTexture", {{"scale", 1, T_FLOAT, nullptr, false, 0}}},
      {"SpectralConstantTexture",
       {{"gaussian", 1, T_MSG, "GaussianSpectralConstant", false, 1},
        {"tabulated", 2, T_MSG, "TabulatedSpectralConstant", false, 1},
        {"neutral", 3, T_MSG, "NeutralSpectralConstant", false, 1},
        {"from_light_source_library", 4, T_MSG, "FromLightSourceLibrary", false, 1}}},
      {"GaussianSpectralConstant",
       {{"peak_value", 1, T_FLOAT, nullptr, false, 0}, {"center_wavelength", 2, T_FLOAT, nullptr, false, 0},
        {"width", 3, T_FLOAT, nullptr, false, 0}}},
      {"TabulatedSpectralConstant",
       {{"wavelengths", 1, T_FLOAT, nullptr, true, 0}, {"values", 2, T_FLOAT, nullptr, true, 0}}},
      {"NeutralSpectralConstant", {{"reflectance", 1, T_FLOAT, nullptr, false, 0}}},
      {"FromLightSourceLibrary", {{"light_source_name", 1, T_STRING, nullptr, false, 0}}},
      {"SpectralCheckerTexture",
       {{"odd", 1, T_MSG, "SpectralConstantTexture", false, 0}, {"even", 2, T_MSG, "SpectralConstantTexture", false, 0}}},
      {"Material",
       {{"name", 1, T_STRING, nullptr, false, 0}, {"type", 2, T_ENUM, "MaterialType", false, 0},
        {"dielectric", 3, T_MSG, "DielectricMaterial", false, 1}, {"diffuselight", 4, T_MSG, "DiffuseLightMaterial", false, 1},
        {"isotropic", 5, T_MSG, "IsotropicMaterial", false, 1}, {"lambert", 6, T_MSG, "LambertMaterial", false, 1},
        {"metal", 7, T_MSG, "MetalMaterial", false, 1}, {"pbr", 8, T_MSG, "PBRMaterial", false, 1}}},
      {"LambertMaterial",
       {{"albedo", 1, T_MSG, "Texture", false, 1}, {"spectral_albedo", 2, T_MSG, "SpectralConstantTexture", false, 1}}},
      {"DielectricMaterial",
       {{"refidx", 1, T_FLOAT, nullptr, false, 1}, {"spectral_refidx", 2, T_MSG, "SpectralConstantTexture", false, 1},
        {"compute_beer_lambert_attenuation", 3, T_BOOL, nullptr, false, 0},
        {"absorption_coeff", 4, T_MSG, "Vec3", false, 2},
        {"spectral_absorption_coeff", 5, T_MSG, "SpectralConstantTexture", false, 2}}},
      {"DiffuseLightMaterial",
       {{"emit", 1, T_MSG, "Texture", false, 1}, {"spectral_emit", 2, T_MSG, "SpectralConstantTexture", false, 1}}},
      {"IsotropicMaterial",
       {{"albedo", 1, T_MSG, "Texture", false, 1}, {"spectral_albedo", 2, T_MSG, "SpectralConstantTexture", false, 1}}},
      {"MetalMaterial", {{"albedo", 1, T_MSG, "Vec3", false, 0}, {"fuzz", 2, T_FLOAT, nullptr, false, 0}}},
      {"PBRMaterial",
       {{"albedo", 1, T_MSG, "Texture", false, 0}, {"roughness", 2, T_MSG, "Texture", false, 0},
        {"metalness", 3, T_MSG, "Texture", false, 0}, {"normal_map", 4, T_MSG, "Texture", false, 0},
        {"sss", 5, T_MSG, "Texture", false, 0}, {"sss_radius", 6, T_FLOAT, nullptr, false, 0}}},
      {"Triangle",
       {{"vertex0", 1, T_MSG, "Vec3", false, 0}, {"vertex1", 2, T_MSG, "Vec3", false, 0}, {"vertex2", 3, T_MSG, "Vec3", false, 0},
        {"uv0", 4, T_MSG, "Vec2", false, 0}, {"uv1", 5, T_MSG, "Vec2", false, 0}, {"uv2", 6, T_MSG, "Vec2", false, 0},
        {"normal0", 7, T_MSG, "Vec3", false, 0}, {"normal1", 8, T_MSG, "Vec3", false, 0}, {"normal2", 9, T_MSG, "Vec3", false, 0},
        {"material_name", 10, T_STRING, nullptr, false, 0}, {"operator", 11, T_ENUM, "GeometryOperator", false, 0},
        {"displace", 12, T_MSG, "DisplaceOperator", false, 1}}},
      {"Sphere",
       {{"center", 1, T_MSG, "Vec3", false, 0}, {"radius", 2, T_FLOAT, nullptr, false, 0},
        {"material_name", 3, T_STRING, nullptr, false, 0}}},
      {"SceneObjects", {{"triangles", 1, T_MSG, "Triangle", true, 0}, {"spheres", 2, T_MSG, "Sphere", true, 0}}},
      // map<string, V> fields are repeated entry messages {key = 1, value = 2}
      {"MaterialsEntry", {{"key", 1, T_STRING, nullptr, false, 0}, {"value", 2, T_MSG, "Material", false, 0}}},
      {"ImageTexturesEntry",
       {{"key", 1, T_STRING, nullptr, false, 0}, {"value", 2, T_MSG, "ImageTextureMetadata", false, 0}}},
      {"Scene",
       {{"name", 1, T_STRING, nullptr, false, 0}, {"version", 2, T_STRING, nullptr, false, 0},
        {"colour_representation", 3, T_ENUM, "ColourRepresentation", false, 0}, {"camera", 4, T_MSG, "Camera", false, 0},
        {"materials", 5, T_MSG, "MaterialsEntry", true, 0}, {"image_textures", 6, T_MSG, "ImageTexturesEntry", true, 0},
        {"displacement_maps", 7, T_MSG, "ImageTexturesEntry", true, 0}, {"objects", 8, T_MSG, "SceneObjects", false, 0},
        {"stream_triangles", 9, T_BOOL, nullptr, false, 0}, {"total_triangles", 10, T_UINT64, nullptr, false, 0},
        {"spectral_background", 11, T_MSG, "TabulatedSpectralConstant", false, 0}}},
  };
  return m;
}

const MsgDef* msg_def(const char* name) {
  for (const auto& d : messages())
    if (!strcmp(d.name, name)) return &d;
  return nullptr;
}

const EnumDef* enum_def(const char* name) {
  for (const auto& d : enums())
    if (!strcmp(d.name, name)) return &d;
  return nullptr;
}

struct PMsg;
struct PVal {
  double num = 0;   // T_FLOAT (already rounded to float32) / T_DOUBLE
  uint64_t u = 0;   // ints, bools, enum numbers
  std::string s;    // strings
  std::shared_ptr<PMsg> m;
};

struct PMsg {
  const MsgDef* def;
  std::vector<std::vector<PVal>> f;  // per field of def, in occurrence order
  explicit PMsg(const MsgDef* d) : def(d), f(d->fields.size()) {}

  bool has(const char* name) const {
    int i = def->find(name);
    return i >= 0 && !f[i].empty();
  }
  const PVal* get(const char* name) const {
    int i = def->find(name);
    return (i >= 0 && !f[i].empty()) ? &f[i].back() : nullptr;
  }
  const PMsg* msg(const char* name) const {
    const PVal* v = get(name);
    return v ? v->m.get() : nullptr;
  }
  // proto3 getters: zero value when unset (GetX() on a nil message included)
  double num(const char* name) const { const PVal* v = get(name); return v ? v->num : 0.0; }
  uint64_t u(const char* name) const { const PVal* v = get(name); return v ? v->u : 0; }
  std::string str(const char* name) const { const PVal* v = get(name); return v ? v->s : std::string(); }
  const std::vector<PVal>& all(const char* name) const { return f[def->find(name)]; }
  // which member of a oneof group is set ("" = none)
  const char* oneof(int group) const {
    for (size_t i = 0; i < def->fields.size(); i++)
      if (def->fields[i].oneof == group && !f[i].empty()) return def->fields[i].name;
    return "";
  }
};

double getf(const PMsg* m, const char* name) { return m ? m->num(name) : 0.0; }

// ------------------------------------------------------------------ text format
// prototext.Unmarshal (google.golang.org/protobuf/encoding/prototext): unknown fields,
// a repeated non-repeated field and two members of one oneof are errors.
constexpr int kMaxNesting = 64;  // transport.proto nests 8 deep; deeper input is malformed

struct TextParser {
  const char* p;
  const char* e;
  int line = 1;
  int depth = 0;

  [[noreturn]] void err(const std::string& m) {
    invalid("pbtxt line " + std::to_string(line) + ": " + m);
  }
  void skip_ws() {
    while (p < e) {
      if (*p == '\n') { line++; p++; }
      else if (isspace((unsigned char)*p)) p++;
      else if (*p == '#') { while (p < e && *p != '\n') p++; }
      else break;
    }
  }
  bool peek(char c) { skip_ws(); return p < e && *p == c; }
  bool accept(char c) { if (peek(c)) { p++; return true; } return false; }
  void expect(char c) { if (!accept(c)) err(std::string("expected '") + c + "'"); }
  std::string ident() {
    skip_ws();
    const char* b = p;
    if (p < e && (isalpha((unsigned char)*p) || *p == '_')) {
      p++;
      while (p < e && (isalnum((unsigned char)*p) || *p == '_')) p++;
    }
    if (p == b) err("expected an identifier");
    return std::string(b, p);
  }
  // a scalar token: number / identifier text (not a string)
  std::string token() {
    skip_ws();
    const char* b = p;
    while (p < e && (isalnum((unsigned char)*p) || *p == '_' || *p == '.' || *p == '-' || *p == '+')) p++;
    if (p == b) err("expected a value");
    return std::string(b, p);
  }
  std::string string_lit() {
    std::string out;
    bool any = false;
    for (;;) {
      skip_ws();
      if (p >= e || (*p != '"' && *p != '\'')) break;
      any = true;
      const char q = *p++;
      while (p < e && *p != q) {
        if (*p == '\n') err("newline in string");
        if (*p != '\\') { out += *p++; continue; }
        if (++p >= e) err("bad escape");
        const char c = *p++;
        switch (c) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'r': out += '\r'; break;
          case 'a': out += '\a'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'v': out += '\v'; break;
          case '\\': case '\'': case '"': case '?': out += c; break;
          case 'x': {
            int v = 0, n = 0;
            while (n < 2 && p < e && isxdigit((unsigned char)*p)) { v = v * 16 + (isdigit((unsigned char)*p) ? *p - '0' : (tolower(*p) - 'a' + 10)); p++; n++; }
            if (!n) err("bad \\x escape");
            out += (char)v;
            break;
          }
          default:
            if (c >= '0' && c <= '7') {
              int v = c - '0', n = 1;
              while (n < 3 && p < e && *p >= '0' && *p <= '7') { v = v * 8 + (*p++ - '0'); n++; }
              out += (char)v;
            } else {
              err(std::string("unsupported escape \\") + c);
            }
        }
      }
      if (p >= e) err("unterminated string");
      p++;
    }
    if (!any) err("expected a string");
    return out;
  }

  PVal scalar(const FieldDef& fd) {
    PVal v;
    switch (fd.type) {
      case T_STRING: v.s = string_lit(); break;
      case T_FLOAT:
      case T_DOUBLE: {
        std::string t = token();
        std::string l = t;
        std::transform(l.begin(), l.end(), l.begin(), ::tolower);
        bool neg = !l.empty() && l[0] == '-';
        std::string body = neg ? l.substr(1) : l;
        if (body == "inf" || body == "infinity") { v.num = neg ? -__builtin_inf() : __builtin_inf(); break; }
        if (body == "nan") { v.num = __builtin_nan(""); break; }
        if (!body.empty() && (body.back() == 'f') && body.find('x') == std::string::npos) t.pop_back();
        double d;
        if (!go_parse_float(t, fd.type == T_FLOAT, &d)) err("invalid value for " + std::string(fd.name) + ": " + t);
        v.num = d;
        break;
      }
      case T_UINT32:
      case T_UINT64: {
        std::string t = token();
        char* end = nullptr;
        errno = 0;
        if (t.empty() || t[0] == '-') err("invalid value for " + std::string(fd.name) + ": " + t);
        unsigned long long x = strtoull(t.c_str(), &end, 0);
        if (*end || errno == ERANGE || (fd.type == T_UINT32 && x > 0xFFFFFFFFull))
          err("invalid value for " + std::string(fd.name) + ": " + t);
        v.u = x;
        break;
      }
      case T_BOOL: {
        std::string t = token();
        if (t == "true" || t == "True" || t == "t" || t == "1") v.u = 1;
        else if (t == "false" || t == "False" || t == "f" || t == "0") v.u = 0;
        else err("invalid value for " + std::string(fd.name) + ": " + t);
        break;
      }
      case T_ENUM: {
        std::string t = token();
        const EnumDef* ed = enum_def(fd.sub);
        bool found = false;
        for (auto& kv : ed->values)
          if (t == kv.first) { v.u = (uint64_t)kv.second; found = true; }
        if (!found) {
          char* end = nullptr;
          long long x = strtoll(t.c_str(), &end, 10);
          if (t.empty() || *end) err("invalid value for enum " + std::string(fd.sub) + ": " + t);
          v.u = (uint64_t)x;  // proto3 enums are open: unknown numbers are kept
        }
        break;
      }
      case T_MSG: break;
    }
    return v;
  }

  void message_body(PMsg& m, char close) {
    for (;;) {
      skip_ws();
      if (close ? peek(close) : p >= e) break;
      if (p >= e) err("unexpected end of input");
      if (*p == '[') err("extension / Any fields are not part of transport.proto");
      const std::string name = ident();
      const int fi = m.def->find(name);
      if (fi < 0) err("unknown field \"" + name + "\" in " + m.def->name);
      const FieldDef& fd = m.def->fields[fi];
      bool list = false;
      if (fd.type == T_MSG) {
        if (accept(':')) list = peek('[');
      } else {
        expect(':');
        list = peek('[');
      }
      if (list && !fd.repeated) err("list value for non-repeated field " + name);
      if (list) expect('[');
      bool first = true;
      for (;;) {
        if (list) {
          if (accept(']')) break;
          if (!first) expect(',');
          if (accept(']')) err("trailing ','");
        }
        first = false;
        if (!fd.repeated && !m.f[fi].empty()) err("non-repeated field \"" + name + "\" is repeated");
        if (fd.oneof) {
          for (size_t j = 0; j < m.def->fields.size(); j++)
            if ((int)j != fi && m.def->fields[j].oneof == fd.oneof && !m.f[j].empty())
              err("field \"" + name + "\" is in a oneof whose member \"" + m.def->fields[j].name + "\" is already set");
        }
        PVal v;
        if (fd.type == T_MSG) {
          char open = 0;
          if (accept('{')) open = '}';
          else if (accept('<')) open = '>';
          else err("expected '{' for message field " + name);
          v.m = std::make_shared<PMsg>(msg_def(fd.sub));
          if (++depth > kMaxNesting) err("messages nested too deeply");
          message_body(*v.m, open);
          depth--;
          expect(open);
        } else {
          v = scalar(fd);
        }
        m.f[fi].push_back(std::move(v));
        if (!list) break;
      }
      if (!accept(',')) accept(';');
    }
  }
};

// ------------------------------------------------------------------ wire format
// proto.Unmarshal: unknown fields are skipped, a repeated singular scalar keeps the
// last value, a repeated singular message merges, the last oneof member set wins,
// repeated scalars may be packed or not.
struct WireParser {
  const uint8_t* p;
  const uint8_t* e;
  int depth = 0;

  [[noreturn]] void err(const std::string& m) { invalid("izpi (binary protobuf): " + m); }
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 64; s += 7) {
      if (p >= e) err("truncated varint");
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7F) << s;
      if (!(b & 0x80)) return v;
    }
    err("varint too long");
  }
  uint32_t fixed32() { if (e - p < 4) err("truncated fixed32"); uint32_t v; memcpy(&v, p, 4); p += 4; return v; }
  uint64_t fixed64() { if (e - p < 8) err("truncated fixed64"); uint64_t v; memcpy(&v, p, 8); p += 8; return v; }

  static void merge(PMsg& dst, const PMsg& src) {
    for (size_t i = 0; i < src.f.size(); i++) {
      if (src.f[i].empty()) continue;
      const FieldDef& fd = dst.def->fields[i];
      if (fd.oneof)
        for (size_t j = 0; j < dst.f.size(); j++)
          if (j != i && dst.def->fields[j].oneof == fd.oneof) dst.f[j].clear();
      if (fd.repeated) {
        for (auto& v : src.f[i]) dst.f[i].push_back(v);
      } else if (fd.type == T_MSG && !dst.f[i].empty()) {
        auto merged = std::make_shared<PMsg>(*dst.f[i].back().m);
        merge(*merged, *src.f[i].back().m);
        dst.f[i].back().m = merged;
      } else {
        dst.f[i] = {src.f[i].back()};
      }
    }
  }

  void put(PMsg& m, int fi, PVal v) {
    const FieldDef& fd = m.def->fields[fi];
    if (fd.oneof)
      for (size_t j = 0; j < m.f.size(); j++)
        if ((int)j != fi && m.def->fields[j].oneof == fd.oneof) m.f[j].clear();
    if (fd.repeated) { m.f[fi].push_back(std::move(v)); return; }
    if (fd.type == T_MSG && !m.f[fi].empty()) {
      auto merged = std::make_shared<PMsg>(*m.f[fi].back().m);
      merge(*merged, *v.m);
      m.f[fi].back().m = merged;
      return;
    }
    m.f[fi] = {std::move(v)};
  }

  PVal from_bits(const FieldDef& fd, uint64_t raw, int wt) {
    PVal v;
    switch (fd.type) {
      case T_FLOAT: {
        if (wt != 5) err(std::string("wrong wire type for ") + fd.name);
        float f; uint32_t b = (uint32_t)raw; memcpy(&f, &b, 4); v.num = (double)f; break;
      }
      case T_DOUBLE: {
        if (wt != 1) err(std::string("wrong wire type for ") + fd.name);
        double d; memcpy(&d, &raw, 8); v.num = d; break;
      }
      case T_UINT32: case T_UINT64: case T_BOOL: case T_ENUM:
        if (wt != 0) err(std::string("wrong wire type for ") + fd.name);
        v.u = fd.type == T_UINT32 ? (uint32_t)raw : fd.type == T_BOOL ? (raw != 0) : fd.type == T_ENUM ? (uint64_t)(int64_t)(int32_t)raw : raw;
        break;
      default: err("bad scalar");
    }
    return v;
  }

  void parse(PMsg& m) {
    while (p < e) {
      const uint64_t key = varint();
      const int num = (int)(key >> 3), wt = (int)(key & 7);
      if (num <= 0) err("invalid field number");
      const int fi = m.def->find_num(num);
      if (wt == 3 || wt == 4) err("groups are not supported");
      if (fi < 0) {  // unknown field: skip
        if (wt == 0) varint();
        else if (wt == 1) fixed64();
        else if (wt == 5) fixed32();
        else if (wt == 2) { uint64_t n = varint(); if ((uint64_t)(e - p) < n) err("truncated field"); p += n; }
        else err("bad wire type");
        continue;
      }
      const FieldDef& fd = m.def->fields[fi];
      if (wt == 2) {
        const uint64_t n = varint();
        if ((uint64_t)(e - p) < n) err("truncated field");
        const uint8_t* end = p + n;
        if (fd.type == T_STRING) {
          PVal v; v.s.assign((const char*)p, n); p = end; put(m, fi, std::move(v));
        } else if (fd.type == T_MSG) {
          PVal v; v.m = std::make_shared<PMsg>(msg_def(fd.sub));
          if (depth + 1 > kMaxNesting) err("messages nested too deeply");
          WireParser sub{p, end, depth + 1}; sub.parse(*v.m); p = end;
          put(m, fi, std::move(v));
        } else if (fd.repeated) {  // packed
          while (p < end) {
            uint64_t raw = fd.type == T_FLOAT ? fixed32() : fd.type == T_DOUBLE ? fixed64() : varint();
            put(m, fi, from_bits(fd, raw, fd.type == T_FLOAT ? 5 : fd.type == T_DOUBLE ? 1 : 0));
          }
          if (p != end) err("packed field overruns");
        } else {
          err(std::string("wrong wire type for ") + fd.name);
        }
      } else {
        uint64_t raw = wt == 0 ? varint() : wt == 1 ? fixed64() : wt == 5 ? fixed32() : (err("bad wire type"), 0);
        put(m, fi, from_bits(fd, raw, wt));
      }
    }
  }
};

// proto.Marshal of a field tree (google.golang.org/protobuf): fields in field-number
// order, repeated scalars packed (proto3), repeated messages and map entries in
// occurrence order, proto3 scalars at their zero value omitted unless they are a oneof
// member (presence) or a map entry's key.
struct WireWriter {
  std::string out;
  void varint(uint64_t v) {
    do {
      uint8_t b = v & 0x7F;
      v >>= 7;
      out.push_back((char)(b | (v ? 0x80 : 0)));
    } while (v);
  }
  void key(int num, int wt) { varint((uint64_t)num << 3 | (uint64_t)wt); }
  void f32(double x) { const float f = (float)x; uint32_t b; memcpy(&b, &f, 4); out.append((const char*)&b, 4); }
  void f64(double x) { uint64_t b; memcpy(&b, &x, 8); out.append((const char*)&b, 8); }
  static bool zero(const FieldDef& fd, const PVal& v) {
    switch (fd.type) {
      case T_FLOAT: { const float f = (float)v.num; uint32_t b; memcpy(&b, &f, 4); return b == 0; }  // -0 is kept
      case T_DOUBLE: { uint64_t b; memcpy(&b, &v.num, 8); return b == 0; }
      case T_STRING: return v.s.empty();
      case T_MSG: return false;
      default: return v.u == 0;
    }
  }
  void scalar(const FieldDef& fd, const PVal& v) {
    if (fd.type == T_FLOAT) f32(v.num);
    else if (fd.type == T_DOUBLE) f64(v.num);
    else varint(fd.type == T_ENUM ? (uint64_t)(int64_t)(int32_t)v.u : v.u);
  }
  void msg(const PMsg& m) {
    std::vector<int> order(m.def->fields.size());
    for (size_t i = 0; i < order.size(); i++) order[i] = (int)i;
    std::sort(order.begin(), order.end(), [&](int a, int b) { return m.def->fields[a].num < m.def->fields[b].num; });
    const bool entry = strstr(m.def->name, "Entry") != nullptr;
    for (int fi : order) {
      const FieldDef& fd = m.def->fields[fi];
      const std::vector<PVal>& vals = m.f[fi];
      if (vals.empty()) continue;
      if (fd.repeated && fd.type != T_MSG && fd.type != T_STRING) {  // packed
        WireWriter w;
        for (const PVal& v : vals) w.scalar(fd, v);
        key(fd.num, 2);
        varint(w.out.size());
        out += w.out;
        continue;
      }
      const size_t n = fd.repeated ? vals.size() : 1;
      for (size_t k = 0; k < n; k++) {
        const PVal& v = fd.repeated ? vals[k] : vals.back();
        if (!fd.repeated && !fd.oneof && !entry && zero(fd, v)) continue;
        if (fd.type == T_MSG || fd.type == T_STRING) {
          std::string payload;
          if (fd.type == T_MSG) { WireWriter w; w.msg(*v.m); payload.swap(w.out); } else payload = v.s;
          key(fd.num, 2);
          varint(payload.size());
          out += payload;
        } else {
          key(fd.num, fd.type == T_FLOAT ? 5 : fd.type == T_DOUBLE ? 1 : 0);
          scalar(fd, v);
        }
      }
    }
  }
};

// ================================================================ transport.ToScene
struct LightSpd { std::vector<double> values; };

// spectral.NewBlackbodySPD (spectral.go:275-318): c1/c2 are exact Go constant
// expressions (generated), the rest float64 in Go's evaluation order.
std::vector<double> blackbody(double temperature) {
  std::vector<double> v(IZPI_CIE_N);
  double maxv = 0.0;
  for (int i = 0; i < IZPI_CIE_N; i++) {
    const double wm = izpi_cie_wavelengths[i] * 1e-9;
    const double w5 = wm * wm * wm * wm * wm;
    const double ex = IZPI_BLACKBODY_C2 / (wm * temperature);
    v[i] = ex > 700 ? 0.0 : IZPI_BLACKBODY_C1 / (w5 * (gm::exp(ex) - 1.0));
    if (v[i] > maxv) maxv = v[i];
  }
  if (maxv > 0)
    for (auto& x : v) x /= maxv;
  return v;
}

}  // namespace

// ---- the opaque handles ------------------------------------------------------
struct izpi_proto_scene {
  std::shared_ptr<PMsg> root;
  std::map<std::string, std::pair<uint32_t, uint32_t>> image_dims;
  std::map<std::string, std::vector<double>> images;            // filename -> W*H*4 float64 NRGBA
  std::vector<std::pair<std::string, std::vector<izpi_tri_in>>> streamed;  // transport.go:574-583
  std::vector<std::string> image_files;                          // image_textures values' filenames
  std::string name, version, warnings;
  // built by izpi_scene_to_input
  std::vector<izpi_tri_in> tris;
  std::vector<izpi_sphere_in> spheres;
  std::vector<izpi_material> mats;
  std::vector<izpi_texture> texs;
  std::vector<double> texels, spd_wl, spd_val;
  std::map<std::string, uint64_t> texel_offset;
  std::vector<std::string> mat_names;
  izpi_scene_input input;
};

namespace {

struct Converter {
  izpi_proto_scene& s;
  bool spectral;

  int add_tex(const izpi_texture& t) { s.texs.push_back(t); return (int)s.texs.size() - 1; }
  static izpi_texture blank(uint32_t kind) { izpi_texture t; memset(&t, 0, sizeof t); t.kind = kind; return t; }

  int constant(double r, double g, double b) {
    izpi_texture t = blank(IZPI_TEX_CONSTANT);
    t.value[0] = r; t.value[1] = g; t.value[2] = b;
    return add_tex(t);
  }
  int tabulated(const std::vector<double>& wl, const std::vector<double>& vals) {
    if (wl.size() != vals.size() || wl.empty())
      invalid("tabulated SPD with " + std::to_string(wl.size()) + " wavelengths and " + std::to_string(vals.size()) +
              " values (the reference indexes values by wavelength)");
    izpi_texture t = blank(IZPI_TEX_SPECTRAL_TABULATED);
    t.spd_offset = (uint32_t)s.spd_wl.size();
    t.spd_count = (uint32_t)wl.size();
    s.spd_wl.insert(s.spd_wl.end(), wl.begin(), wl.end());
    s.spd_val.insert(s.spd_val.end(), vals.begin(), vals.end());
    return add_tex(t);
  }
  // texture.NewSpectralNeutral (spectral_constant.go:83-96)
  int neutral(double r) {
    std::vector<double> wl, v;
    for (int w = 380; w <= 750; w += 10) { wl.push_back((double)w); v.push_back(r); }
    return tabulated(wl, v);
  }

  // toSceneSpectralTexture (transport.go:440-484)
  int spectral_texture(const PMsg* st) {
    const std::string which = st ? st->oneof(1) : "";
    if (which == "gaussian") {
      const PMsg* g = st->msg("gaussian");
      izpi_texture t = blank(IZPI_TEX_SPECTRAL_GAUSSIAN);
      t.peak = g->num("peak_value"); t.center = g->num("center_wavelength"); t.width_nm = g->num("width");
      return add_tex(t);
    }
    if (which == "tabulated") {
      const PMsg* tb = st->msg("tabulated");
      std::vector<double> wl, v;
      for (auto& x : tb->all("wavelengths")) wl.push_back(x.num);
      for (auto& x : tb->all("values")) v.push_back(x.num);
      return tabulated(wl, v);
    }
    if (which == "neutral") return neutral(st->msg("neutral")->num("reflectance"));
    if (which == "from_light_source_library") {
      const std::string name = st->msg("from_light_source_library")->str("light_source_name");
      const izpi_light_source_entry* hit = nullptr;
      for (int i = 0; i < IZPI_NUM_LIGHT_SOURCES; i++)
        if (name == izpi_light_source_library[i].name) hit = &izpi_light_source_library[i];
      if (!hit) {
        s.warnings += "Light source '" + name + "' not found in library, defaulting to CIE Illuminant A (2856K)\n";
        for (int i = 0; i < IZPI_NUM_LIGHT_SOURCES; i++)
          if (!strcmp("cie_illuminant_a_2856k", izpi_light_source_library[i].name)) hit = &izpi_light_source_library[i];
      }
      std::vector<double> wl(IZPI_CIE_N), v;
      for (int i = 0; i < IZPI_CIE_N; i++) wl[i] = izpi_cie_wavelengths[i];
      if (hit->temperature > 0) v = blackbody(hit->temperature);
      else v.assign(hit->values, hit->values + IZPI_CIE_N);
      return tabulated(wl, v);
    }
    invalid("unknown spectral texture type");
  }

  // toSceneTexture (transport.go:390-438)
  int texture(const PMsg* t) {
    const std::string which = t ? t->oneof(1) : "";
    if (which == "constant") {
      const PMsg* v = t->msg("constant")->msg("value");
      return constant(getf(v, "x"), getf(v, "y"), getf(v, "z"));
    }
    if (which == "image") {
      const std::string fn = t->msg("image")->str("filename");
      auto it = s.images.find(fn);
      if (it == s.images.end()) invalid("texture " + fn + " not found");
      const auto dims = s.image_dims[fn];
      auto off = s.texel_offset.find(fn);
      if (off == s.texel_offset.end()) {
        off = s.texel_offset.emplace(fn, (uint64_t)s.texels.size()).first;
        s.texels.insert(s.texels.end(), it->second.begin(), it->second.end());
      }
      izpi_texture x = blank(IZPI_TEX_IMAGE);
      x.width = dims.first; x.height = dims.second; x.texel_offset = off->second;
      return add_tex(x);
    }
    if (which == "spectral_constant") {  // validated, then the neutral RGB fallback
      spectral_texture(t->msg("spectral_constant"));
      return constant(0.5, 0.5, 0.5);
    }
    if (which == "spectral_checker") return constant(0.5, 0.5, 0.5);
    invalid(std::string("unknown texture type: ") + (which.empty() ? "<nil>" : which));
  }

  static izpi_material blank_mat(uint32_t kind) {
    izpi_material m;
    memset(&m, 0, sizeof m);
    m.kind = kind;
    m.albedo_tex = m.spectral_tex = m.normal_tex = m.roughness_tex = m.metalness_tex = m.absorb_tex = -1;
    return m;
  }

  // toSceneMaterial and its cases (transport.go:134-388); `ok` false = type not converted
  izpi_material material(const PMsg* m, bool* ok) {
    *ok = true;
    const uint64_t type = m ? m->u("type") : 0;
    const std::string mname = m ? m->str("name") : "";
    switch (type) {
      case IZPI_MAT_LAMBERT: {
        const PMsg* l = m->msg("lambert");
        const std::string w = l ? l->oneof(1) : "";
        izpi_material r = blank_mat(IZPI_MAT_LAMBERT);
        if (w == "albedo") r.albedo_tex = texture(l->msg("albedo"));
        else if (w == "spectral_albedo") r.spectral_tex = spectral_texture(l->msg("spectral_albedo"));
        else invalid("lambert material must have either albedo or spectral_albedo");
        return r;
      }
      case IZPI_MAT_DIELECTRIC: {
        const PMsg* d = m->msg("dielectric");
        const std::string ri = d ? d->oneof(1) : "", ab = d ? d->oneof(2) : "";
        izpi_material r = blank_mat(IZPI_MAT_DIELECTRIC);
        if (ri == "refidx") r.ref_idx = d->num("refidx");
        else if (ri == "spectral_refidx") r.spectral_tex = spectral_texture(d->msg("spectral_refidx"));
        else invalid("dielectric material must have either refidx or spectral_refidx");
        double absorb[3] = {0, 0, 0};
        if (ab == "absorption_coeff") {
          const PMsg* a = d->msg("absorption_coeff");
          absorb[0] = getf(a, "x"); absorb[1] = getf(a, "y"); absorb[2] = getf(a, "z");
        } else if (ab == "spectral_absorption_coeff") {
          r.absorb_tex = spectral_texture(d->msg("spectral_absorption_coeff"));
        }
        const bool beer = d->u("compute_beer_lambert_attenuation") != 0;
        if (r.spectral_tex >= 0) {
          // NewSpectralColoredDielectric / NewSpectralDielectric(refidx, beer)
          if (r.absorb_tex < 0 && beer) r.flags = IZPI_MATF_BEER_LAMBERT;
        } else if (absorb[0] != 0 || absorb[1] != 0 || absorb[2] != 0) {
          r.flags = IZPI_MATF_BEER_LAMBERT;  // NewColoredDielectric
        }
        // the RGB absorption is kept as the reference keeps it (zero for plain dielectrics)
        r.rgb[0] = absorb[0]; r.rgb[1] = absorb[1]; r.rgb[2] = absorb[2];
        return r;
      }
      case IZPI_MAT_DIFFUSE_LIGHT: {
        const PMsg* l = m->msg("diffuselight");
        const std::string w = l ? l->oneof(1) : "";
        izpi_material r = blank_mat(IZPI_MAT_DIFFUSE_LIGHT);
        if (w == "emit") r.albedo_tex = texture(l->msg("emit"));
        else if (w == "spectral_emit") r.spectral_tex = spectral_texture(l->msg("spectral_emit"));
        else invalid("diffuse light material must have either emit or spectral_emit");
        return r;
      }
      case IZPI_MAT_METAL: {
        const PMsg* mt = m->msg("metal");
        const PMsg* a = mt ? mt->msg("albedo") : nullptr;
        izpi_material r = blank_mat(IZPI_MAT_METAL);
        r.rgb[0] = getf(a, "x"); r.rgb[1] = getf(a, "y"); r.rgb[2] = getf(a, "z");
        r.fuzz = getf(mt, "fuzz");
        return r;
      }
      case 3: {  // ISOTROPIC (transport.go:264-289)
        const PMsg* l = m->msg("isotropic");
        const std::string w = l ? l->oneof(1) : "";
        if (w == "albedo") {
          izpi_material r = blank_mat(IZPI_MAT_ISOTROPIC);
          r.albedo_tex = texture(l->msg("albedo"));
          return r;
        }
        if (w == "spectral_albedo") {
          spectral_texture(l->msg("spectral_albedo"));
          invalid("spectral isotropic materials not yet implemented");
        }
        invalid("isotropic material must have either albedo or spectral_albedo");
      }
      case IZPI_MAT_PBR: {
        const PMsg* pb = m->msg("pbr");
        izpi_material r = blank_mat(IZPI_MAT_PBR);
        const PMsg* alb = pb ? pb->msg("albedo") : nullptr;
        r.albedo_tex = texture(alb);
        r.roughness_tex = texture(pb ? pb->msg("roughness") : nullptr);
        r.metalness_tex = texture(pb ? pb->msg("metalness") : nullptr);
        r.normal_tex = texture(pb ? pb->msg("normal_map") : nullptr);
        texture(pb ? pb->msg("sss") : nullptr);  // required by the reference, unused by PBR.Scatter
        if (spectral) {  // textureToSpectralTexture (transport.go:486-520)
          const izpi_texture a = s.texs[r.albedo_tex];
          if (a.kind == IZPI_TEX_IMAGE) {  // NewSpectralImageFromImage of the image's texels
            izpi_texture si = blank(IZPI_TEX_SPECTRAL_IMAGE);
            si.width = a.width; si.height = a.height; si.texel_offset = a.texel_offset;
            s.texs.push_back(si);
            r.spectral_tex = (int32_t)s.texs.size() - 1;
          } else {
            const double lum = 0.299 * a.value[0] + 0.587 * a.value[1] + 0.114 * a.value[2];
            r.spectral_tex = neutral(lum);
          }
        }
        return r;
      }
      default:
        *ok = false;  // unconverted types are silently skipped (transport.go:145-213)
        return blank_mat(0);
    }
  }

  void tri(const PMsg* t, uint32_t mat, izpi_tri_in& o) {
    memset(&o, 0, sizeof o);
    const char* vn[3] = {"vertex0", "vertex1", "vertex2"};
    double* vo[3] = {o.v0, o.v1, o.v2};
    for (int k = 0; k < 3; k++) {
      const PMsg* v = t->msg(vn[k]);
      vo[k][0] = getf(v, "x"); vo[k][1] = getf(v, "y"); vo[k][2] = getf(v, "z");
    }
    const char* un[3] = {"uv0", "uv1", "uv2"};
    for (int k = 0; k < 3; k++) {
      const PMsg* uv = t->msg(un[k]);
      o.uv[2 * k] = getf(uv, "u"); o.uv[2 * k + 1] = getf(uv, "v");
    }
    o.material = mat;
  }

  void run(double aspect_override, uint64_t bvh_seed) {
    const PMsg& sc = *s.root;
    s.tris.clear(); s.spheres.clear(); s.mats.clear(); s.texs.clear();
    s.texels.clear(); s.spd_wl.clear(); s.spd_val.clear(); s.texel_offset.clear(); s.mat_names.clear();
    // materials: map entries (last duplicate key wins), registered under Material.name
    std::vector<std::string> keys;
    std::map<std::string, const PMsg*> by_key;
    for (auto& e : sc.all("materials")) {
      const std::string k = e.m->str("key");
      if (!by_key.count(k)) keys.push_back(k);
      by_key[k] = e.m->msg("value");
    }
    std::map<std::string, uint32_t> by_name;
    std::vector<std::string> errs;
    for (auto& k : keys) {
      const PMsg* m = by_key[k];
      bool ok = false;
      izpi_material r;
      try {
        r = material(m, &ok);
      } catch (const Fail& f) {
        if (f.code != IZPI_ERR_INVALID) throw;
        errs.push_back(f.msg);
        continue;
      }
      if (!ok) continue;
      const std::string name = m->str("name");
      s.mats.push_back(r);
      s.mat_names.push_back(name);
      by_name[name] = (uint32_t)s.mats.size() - 1;
    }
    if (!errs.empty()) {
      std::string all = "errors converting materials: [";
      for (size_t i = 0; i < errs.size(); i++) all += (i ? " " : "") + errs[i];
      invalid(all + "]");
    }
    auto lookup = [&](const std::string& n) {
      auto it = by_name.find(n);
      if (it == by_name.end()) invalid("material " + n + " not found");
      return it->second;
    };
    const PMsg* objs = sc.msg("objects");
    if (objs) {
      for (auto& t : objs->all("triangles")) {
        const PMsg* tm = t.m.get();
        const uint32_t mat = lookup(tm->str("material_name"));
        if (tm->u("operator") == 1)
          fail(IZPI_ERR_UNSUPPORTED, "triangle DISPLACE operator (displacement maps are outside the GPU path)");
        izpi_tri_in o;
        tri(tm, mat, o);
        s.tris.push_back(o);
      }
    }
    for (auto& group : s.streamed) {
      const uint32_t mat = lookup(group.first);
      for (auto o : group.second) { o.material = mat; s.tris.push_back(o); }
    }
    if (objs) {
      for (auto& sp : objs->all("spheres")) {
        const PMsg* sm = sp.m.get();
        izpi_sphere_in o;
        memset(&o, 0, sizeof o);
        o.material = lookup(sm->str("material_name"));
        const PMsg* c = sm->msg("center");
        o.center[0] = getf(c, "x"); o.center[1] = getf(c, "y"); o.center[2] = getf(c, "z");
        o.radius = sm->num("radius");
        s.spheres.push_back(o);
      }
    }
    // camera (transport.go:522-549)
    izpi_scene_input& in = s.input;
    memset(&in, 0, sizeof in);
    const PMsg* cam = sc.msg("camera");
    const char* vn[3] = {"lookfrom", "lookat", "vup"};
    double* vo[3] = {in.camera.look_from, in.camera.look_at, in.camera.vup};
    for (int k = 0; k < 3; k++) {
      const PMsg* v = cam ? cam->msg(vn[k]) : nullptr;
      vo[k][0] = getf(v, "x"); vo[k][1] = getf(v, "y"); vo[k][2] = getf(v, "z");
    }
    in.camera.vfov = getf(cam, "vfov");
    in.camera.aspect = getf(cam, "aspect");
    in.camera.aperture = getf(cam, "aperture");
    in.camera.focus_dist = getf(cam, "focusdist");
    in.camera.time0 = getf(cam, "time0");
    in.camera.time1 = getf(cam, "time1");
    in.camera.exposure = getf(cam, "exposure");
    in.num_tris = (uint32_t)s.tris.size();
    in.num_spheres = (uint32_t)s.spheres.size();
    in.num_materials = (uint32_t)s.mats.size();
    in.num_textures = (uint32_t)s.texs.size();
    in.num_spd = (uint32_t)s.spd_wl.size();
    in.num_texels = s.texels.size();
    in.tris = s.tris.empty() ? nullptr : s.tris.data();
    in.spheres = s.spheres.empty() ? nullptr : s.spheres.data();
    in.materials = s.mats.empty() ? nullptr : s.mats.data();
    in.textures = s.texs.empty() ? nullptr : s.texs.data();
    in.texels = s.texels.empty() ? nullptr : s.texels.data();
    in.spd_wavelengths = s.spd_wl.empty() ? nullptr : s.spd_wl.data();
    in.spd_values = s.spd_val.empty() ? nullptr : s.spd_val.data();
    in.aspect_override = aspect_override;
    in.bvh_seed = bvh_seed;
  }
};

int finish_parse(std::shared_ptr<PMsg> root, izpi_proto_scene** out) {
  auto* s = new izpi_proto_scene();
  s->root = std::move(root);
  s->name = s->root->str("name");
  s->version = s->root->str("version");
  for (auto& e : s->root->all("image_textures")) {
    const PMsg* v = e.m->msg("value");
    s->image_files.push_back(v ? v->str("filename") : std::string());
  }
  memset(&s->input, 0, sizeof s->input);
  *out = s;
  return IZPI_OK;
}

}  // namespace

// ===================================================================== Wavefront OBJ
struct izpi_obj {
  struct VI { int64_t v, vt, vn; };
  struct Face { std::vector<VI> v; };
  struct Group { bool null = false; std::string name, material; uint32_t face_type = 0; std::vector<Face> faces; };
  struct Mtl {
    std::string name;
    std::vector<double> kd, ka, ks;
    double ns = 0, ni = 0, d = 0;
    int64_t sharpness = 0, illum = 0;
  };
  bool ignore_materials = false, ignore_normals = false, ignore_textures = false, has_normals = false, has_uv = false;
  double centre[3] = {0, 0, 0};
  std::string name;
  std::vector<double> v, vn, vt;  // xyz, xyz, uv
  std::map<std::string, Mtl> mtl;
  std::vector<Group> groups;
};

namespace {

std::vector<double> parse_floats(const std::vector<std::string>& t, size_t from) {
  std::vector<double> r;
  for (size_t i = from; i < t.size(); i++) {
    double d;
    if (!go_parse_float(t[i], false, &d)) invalid("strconv.ParseFloat: parsing \"" + t[i] + "\": invalid syntax");
    r.push_back(d);
  }
  return r;
}

// parseMaterialFile (wavefront.go:522-625)
std::map<std::string, izpi_obj::Mtl> parse_mtl(const std::string& file) {
  FILE* f = fopen(file.c_str(), "rb");
  if (!f) invalid("open " + file + ": no such file");
  std::string text;
  char buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) text.append(buf, n);
  fclose(f);
  std::map<std::string, izpi_obj::Mtl> lib;
  izpi_obj::Mtl cur;
  bool have = false;
  auto need = [&]() { if (!have) invalid("mtl: property before newmtl in " + file); };
  auto f32 = [&](const std::string& s) {
    double d;
    if (!go_parse_float(s, true, &d)) invalid("strconv.ParseFloat: parsing \"" + s + "\": invalid syntax");
    return d;
  };
  for (const auto& s : scan_lines(text.data(), text.size())) {
    if (s.empty() || has_prefix(s, "#")) continue;
    const auto t = split_space(s);
    auto arg1 = [&]() -> const std::string& { if (t.size() < 2) invalid("mtl: missing value in \"" + s + "\""); return t[1]; };
    if (has_prefix(s, "newmtl")) {
      if (have) lib[cur.name] = cur;
      cur = izpi_obj::Mtl();
      cur.name = arg1();
      have = true;
      continue;
    }
    if (has_prefix(s, "Kd")) { need(); cur.kd = parse_floats(t, 1); continue; }
    if (has_prefix(s, "Ns")) { need(); cur.ns = f32(arg1()); continue; }
    if (has_prefix(s, "Ni")) { need(); cur.ni = f32(arg1()); continue; }
    if (has_prefix(s, "d")) { need(); cur.d = f32(arg1()); continue; }
    if (has_prefix(s, "illum")) {
      need();
      int64_t v;
      if (!go_parse_int32(arg1(), &v)) invalid("strconv.ParseInt: parsing \"" + arg1() + "\": invalid syntax");
      cur.illum = v;
    }
    if (has_prefix(s, "Ka")) { need(); cur.ka = parse_floats(t, 1); continue; }
    if (has_prefix(s, "Ks")) { need(); cur.ks = parse_floats(t, 1); }
  }
  if (!have) invalid("mtl: no newmtl in " + file);
  lib[cur.name] = cur;
  return lib;
}

// NewObjFromReader (wavefront.go:107-233)
izpi_obj* parse_obj(const char* text, uint64_t len, const std::string& dir, uint32_t opts) {
  std::unique_ptr<izpi_obj> o(new izpi_obj());
  o->ignore_materials = (opts & IZPI_OBJ_IGNORE_MATERIALS) != 0;
  o->ignore_normals = (opts & IZPI_OBJ_IGNORE_NORMALS) != 0;
  o->ignore_textures = (opts & IZPI_OBJ_IGNORE_TEXTURES) != 0;
  std::unique_ptr<izpi_obj::Group> cur;
  std::string active;
  for (const auto& s : scan_lines(text, len)) {
    if (s.empty() || has_prefix(s, "#")) continue;
    const auto t = split_space(s);
    if (has_prefix(s, "o")) {
      if (t.size() == 2) o->name = t[1];
      continue;
    }
    if (has_prefix(s, "v ") || has_prefix(s, "vn") || has_prefix(s, "vt")) {
      const auto v = parse_floats(t, 1);
      const bool isv = has_prefix(s, "v "), isn = has_prefix(s, "vn");
      if (v.size() < (isv || isn ? 3u : 2u)) invalid("too few values in \"" + s + "\"");
      if (isv) { o->v.insert(o->v.end(), v.begin(), v.begin() + 3); }
      else if (isn) { o->has_normals = true; o->vn.insert(o->vn.end(), v.begin(), v.begin() + 3); }
      else { o->has_uv = true; o->vt.push_back(v[0]); o->vt.push_back(v[1]); }
      continue;
    }
    if (has_prefix(s, "f")) {
      if (!cur) { cur.reset(new izpi_obj::Group()); cur->name = "default"; }
      cur->face_type = IZPI_OBJ_FACE_POLYGON;
      izpi_obj::Face face;
      for (size_t i = 1; i < t.size(); i++) {  // parseFaceVertex: exactly "a/b/c"
        std::vector<std::string> idx;
        size_t b = 0;
        for (;;) {
          size_t e = t[i].find('/', b);
          idx.push_back(t[i].substr(b, e == std::string::npos ? std::string::npos : e - b));
          if (e == std::string::npos) break;
          b = e + 1;
        }
        if (idx.size() != 3) invalid("invalid face data");
        int64_t n[3];
        for (int k = 0; k < 3; k++)
          if (!go_parse_int32(idx[k], &n[k])) n[k] = 0;  // missing fields are 0
        face.v.push_back(izpi_obj::VI{n[0], n[1], n[2]});
      }
      cur->faces.push_back(std::move(face));
      continue;
    }
    if (has_prefix(s, "mtllib")) {
      if (o->ignore_materials) continue;
      if (t.size() < 2) invalid("mtllib without a file name");
      o->mtl = parse_mtl(dir + "/" + t[1]);
      continue;
    }
    if (has_prefix(s, "usemtl")) {
      if (t.size() < 2) invalid("usemtl without a name");
      active = t[1];
      continue;
    }
    if (has_prefix(s, "g")) {
      if (cur) o->groups.push_back(*cur);
      if (t.size() < 2) invalid("g without a name");
      cur.reset(new izpi_obj::Group());
      cur->name = t[1];
      cur->material = active;
      continue;
    }
  }
  if (cur) o->groups.push_back(*cur);
  else { izpi_obj::Group g; g.null = true; o->groups.push_back(g); }  // "Add pending group" appends nil
  return o.release();
}

template <typename F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const Fail& e) {
    set_host_error(e.msg);
    return e.code;
  } catch (const std::bad_alloc&) {
    set_host_error("out of host memory");
    return IZPI_ERR_INVALID;
  }
}

}  // namespace

extern "C" {

// ---------------------------------------------------------------- transport.Scene
int izpi_scene_parse_text(const char* text, uint64_t len, izpi_proto_scene** out) {
  if (out) *out = nullptr;
  return guarded([&] {
    if (!out || (!text && len)) invalid("null argument");
    auto root = std::make_shared<PMsg>(msg_def("Scene"));
    TextParser tp{text, text + len};
    tp.message_body(*root, 0);
    return finish_parse(root, out);
  });
}

int izpi_scene_parse_binary(const void* buf, uint64_t len, izpi_proto_scene** out) {
  if (out) *out = nullptr;
  return guarded([&] {
    if (!out || (!buf && len)) invalid("null argument");
    auto root = std::make_shared<PMsg>(msg_def("Scene"));
    WireParser wp{(const uint8_t*)buf, (const uint8_t*)buf + len};
    wp.parse(*root);
    return finish_parse(root, out);
  });
}

int izpi_scene_serialize(const izpi_proto_scene* s, void* buf, uint64_t cap, uint64_t* len) {
  return guarded([&] {
    if (!s || !len || (!buf && cap)) invalid("null argument");
    WireWriter w;
    w.msg(*s->root);
    *len = w.out.size();
    if (buf) memcpy(buf, w.out.data(), std::min<uint64_t>(cap, w.out.size()));
    return IZPI_OK;
  });
}

int izpi_scene_info(const izpi_proto_scene* s, izpi_proto_info* out) {
  return guarded([&] {
    if (!s || !out) invalid("null argument");
    memset(out, 0, sizeof *out);
    const PMsg& r = *s->root;
    out->colour_representation = (uint32_t)r.u("colour_representation");
    out->stream_triangles = (uint32_t)r.u("stream_triangles");
    out->total_triangles = r.u("total_triangles");
    const PMsg* objs = r.msg("objects");
    out->num_triangles = objs ? (uint32_t)objs->all("triangles").size() : 0;
    for (auto& g : s->streamed) out->num_streamed_triangles += (uint32_t)g.second.size();
    out->num_spheres = objs ? (uint32_t)objs->all("spheres").size() : 0;
    out->num_materials = (uint32_t)r.all("materials").size();
    out->num_image_textures = (uint32_t)s->image_files.size();
    out->num_displacement_maps = (uint32_t)r.all("displacement_maps").size();
    const PMsg* bg = r.msg("spectral_background");
    out->num_background = bg ? (uint32_t)bg->all("wavelengths").size() : 0;
    out->name = s->name.c_str();
    out->version = s->version.c_str();
    out->warnings = s->warnings.c_str();
    return IZPI_OK;
  });
}

const char* izpi_scene_image_file(const izpi_proto_scene* s, uint32_t i) {
  return (s && i < s->image_files.size()) ? s->image_files[i].c_str() : nullptr;
}

int izpi_scene_set_image(izpi_proto_scene* s, const char* filename, uint32_t width, uint32_t height,
                         const double* rgba) {
  return guarded([&] {
    if (!s || !filename || (!rgba && width && height)) invalid("null argument");
    s->images[filename].assign(rgba, rgba + (size_t)width * height * 4);
    s->image_dims[filename] = {width, height};
    return IZPI_OK;
  });
}

int izpi_scene_add_triangles(izpi_proto_scene* s, const izpi_tri_in* tris, uint64_t n, const char* material_name) {
  return guarded([&] {
    if (!s || !material_name || (!tris && n)) invalid("null argument");
    s->streamed.emplace_back(material_name, std::vector<izpi_tri_in>(tris, tris + n));
    return IZPI_OK;
  });
}

uint32_t izpi_scene_background(const izpi_proto_scene* s, double* wavelengths, double* values, uint32_t max) {
  if (!s) return 0;
  const PMsg* bg = s->root->msg("spectral_background");
  if (!bg) return 0;
  const auto& w = bg->all("wavelengths");
  const auto& v = bg->all("values");
  const uint32_t n = (uint32_t)std::min(w.size(), v.size());
  for (uint32_t i = 0; i < n && i < max; i++) {
    if (wavelengths) wavelengths[i] = w[i].num;
    if (values) values[i] = v[i].num;
  }
  return n;
}

int izpi_scene_to_input(izpi_proto_scene* s, double aspect_override, uint64_t bvh_seed, const izpi_scene_input** out) {
  if (out) *out = nullptr;
  return guarded([&] {
    if (!s || !out) invalid("null argument");
    const bool spectral = s->root->u("colour_representation") == IZPI_COLOUR_SPECTRAL;
    Converter c{*s, spectral};
    s->warnings.clear();
    c.run(aspect_override, bvh_seed);
    *out = &s->input;
    return IZPI_OK;
  });
}

const char* izpi_scene_material_name(const izpi_proto_scene* s, uint32_t i) {
  return (s && i < s->mat_names.size()) ? s->mat_names[i].c_str() : nullptr;
}

void izpi_scene_free(izpi_proto_scene* s) { delete s; }

uint32_t izpi_light_source(const char* name, double* values) {
  if (!name) return 0;
  for (int i = 0; i < IZPI_NUM_LIGHT_SOURCES; i++) {
    if (strcmp(name, izpi_light_source_library[i].name)) continue;
    const izpi_light_source_entry& e = izpi_light_source_library[i];
    if (values) {
      if (e.temperature > 0) {
        const auto v = blackbody(e.temperature);
        memcpy(values, v.data(), sizeof(double) * IZPI_CIE_N);
      } else {
        memcpy(values, e.values, sizeof(double) * IZPI_CIE_N);
      }
    }
    return IZPI_CIE_N;
  }
  return 0;
}

const char* izpi_light_source_name(uint32_t i) {
  return i < (uint32_t)IZPI_NUM_LIGHT_SOURCES ? izpi_light_source_library[i].name : nullptr;
}

// --------------------------------------------------------------------- Wavefront OBJ
int izpi_obj_parse(const char* text, uint64_t len, const char* container_dir, uint32_t options, izpi_obj** out) {
  if (out) *out = nullptr;
  return guarded([&] {
    if (!out || (!text && len)) invalid("null argument");
    *out = parse_obj(text, len, container_dir ? container_dir : ".", options);
    return IZPI_OK;
  });
}

void izpi_obj_free(izpi_obj* o) { delete o; }

int izpi_obj_info_get(const izpi_obj* o, izpi_obj_info* out) {
  return guarded([&] {
    if (!o || !out) invalid("null argument");
    memset(out, 0, sizeof *out);
    out->has_normals = o->has_normals;
    out->has_uv = o->has_uv;
    out->ignore_materials = o->ignore_materials;
    out->ignore_normals = o->ignore_normals;
    out->ignore_textures = o->ignore_textures;
    out->num_groups = (uint32_t)o->groups.size();
    out->num_materials = (uint32_t)o->mtl.size();
    out->num_vertices = o->v.size() / 3;
    out->num_normals = o->vn.size() / 3;
    out->num_uvs = o->vt.size() / 2;
    memcpy(out->centre, o->centre, sizeof o->centre);
    out->object_name = o->name.c_str();
    return IZPI_OK;
  });
}

int izpi_obj_copy_vertices(const izpi_obj* o, double* v, double* vn, double* vt) {
  if (!o) return IZPI_ERR_INVALID;
  if (v && !o->v.empty()) memcpy(v, o->v.data(), o->v.size() * sizeof(double));
  if (vn && !o->vn.empty()) memcpy(vn, o->vn.data(), o->vn.size() * sizeof(double));
  if (vt && !o->vt.empty()) memcpy(vt, o->vt.data(), o->vt.size() * sizeof(double));
  return IZPI_OK;
}

int izpi_obj_group_get(const izpi_obj* o, uint32_t g, izpi_obj_group* out) {
  return guarded([&] {
    if (!o || !out || g >= o->groups.size()) invalid("bad group index");
    const auto& gr = o->groups[g];
    memset(out, 0, sizeof *out);
    out->name = gr.name.c_str();
    out->material = gr.material.c_str();
    out->face_type = gr.face_type;
    out->is_null = gr.null;
    out->num_faces = gr.faces.size();
    for (auto& f : gr.faces) out->num_face_vertices += f.v.size();
    return IZPI_OK;
  });
}

int izpi_obj_copy_faces(const izpi_obj* o, uint32_t g, uint32_t* face_sizes, int64_t* indices) {
  if (!o || g >= o->groups.size()) return IZPI_ERR_INVALID;
  uint64_t k = 0, i = 0;
  for (auto& f : o->groups[g].faces) {
    if (face_sizes) face_sizes[i] = (uint32_t)f.v.size();
    i++;
    for (auto& vi : f.v) {
      if (indices) { indices[k] = vi.v; indices[k + 1] = vi.vt; indices[k + 2] = vi.vn; }
      k += 3;
    }
  }
  return IZPI_OK;
}

int izpi_obj_material_get(const izpi_obj* o, uint32_t i, izpi_obj_material* out) {
  return guarded([&] {
    if (!o || !out || i >= o->mtl.size()) invalid("bad material index");
    auto it = o->mtl.begin();
    std::advance(it, i);
    const auto& m = it->second;
    memset(out, 0, sizeof *out);
    out->name = m.name.c_str();
    out->num_kd = (uint32_t)std::min<size_t>(m.kd.size(), 3);
    out->num_ka = (uint32_t)std::min<size_t>(m.ka.size(), 3);
    out->num_ks = (uint32_t)std::min<size_t>(m.ks.size(), 3);
    for (uint32_t k = 0; k < out->num_kd; k++) out->kd[k] = m.kd[k];
    for (uint32_t k = 0; k < out->num_ka; k++) out->ka[k] = m.ka[k];
    for (uint32_t k = 0; k < out->num_ks; k++) out->ks[k] = m.ks[k];
    out->ns = m.ns; out->ni = m.ni; out->d = m.d;
    out->sharpness = m.sharpness; out->illum = m.illum;
    return IZPI_OK;
  });
}

// Translate / Scale / Rotate (wavefront.go:418-474)
void izpi_obj_translate(izpi_obj* o, double x, double y, double z) {
  if (!o) return;
  o->centre[0] = o->centre[0] + x; o->centre[1] = o->centre[1] + y; o->centre[2] = o->centre[2] + z;
  for (size_t i = 0; i < o->v.size(); i += 3) { o->v[i] += x; o->v[i + 1] += y; o->v[i + 2] += z; }
}

void izpi_obj_scale(izpi_obj* o, double x, double y, double z) {
  if (!o) return;
  const double s[3] = {x, y, z};
  for (size_t i = 0; i < o->v.size(); i += 3)
    for (int k = 0; k < 3; k++) o->v[i + k] = ((o->v[i + k] - o->centre[k]) * s[k]) + o->centre[k];
}

void izpi_obj_rotate(izpi_obj* o, double alpha, double beta, double gamma) {
  if (!o) return;
  const double ca = gm::cos(alpha), sa = gm::sin(alpha), cb = gm::cos(beta), sb = gm::sin(beta);
  const double cg = gm::cos(gamma), sg = gm::sin(gamma);
  const double* c = o->centre;
  for (size_t i = 0; i < o->v.size(); i += 3) {
    const double x = o->v[i] - c[0], y = o->v[i + 1] - c[1], z = o->v[i + 2] - c[2];
    const double x1 = x * cg - y * sg, y1 = x * sg + y * cg, z1 = z;
    const double x2 = x1 * cb + z1 * sb, y2 = y1, z2 = -x1 * sb + z1 * cb;
    const double x3 = x2, y3 = y2 * ca - z2 * sa, z3 = y2 * sa + z2 * ca;
    o->v[i] = x3 + c[0]; o->v[i + 1] = y3 + c[1]; o->v[i + 2] = z3 + c[2];
  }
}

// GroupToTransportTrianglesWithMaterial (wavefront.go:240-312): the first three vertices
// of each face, rounded to proto float32; UVs float32 or zero (WITHOUT_UVS).
int izpi_obj_group_to_triangles(const izpi_obj* o, uint32_t g, uint32_t without_uvs, izpi_tri_in* out, uint64_t max,
                                uint64_t* n) {
  if (n) *n = 0;
  return guarded([&] {
    if (!o || g >= o->groups.size()) invalid("bad group index");
    const auto& gr = o->groups[g];
    if (gr.null) invalid("group is nil (the file has no faces and no groups)");
    if (gr.face_type != IZPI_OBJ_FACE_POLYGON) fail(IZPI_ERR_UNSUPPORTED, "unsupported polygon type");
    if (n) *n = gr.faces.size();
    if (!out) return IZPI_OK;
    if (max < gr.faces.size()) invalid("output too small");
    const uint64_t nv = o->v.size() / 3, nt = o->vt.size() / 2;
    for (size_t i = 0; i < gr.faces.size(); i++) {
      const auto& f = gr.faces[i];
      if (f.v.size() < 3) invalid("face with fewer than 3 vertices");
      izpi_tri_in& t = out[i];
      memset(&t, 0, sizeof t);
      double* vo[3] = {t.v0, t.v1, t.v2};
      for (int k = 0; k < 3; k++) {
        const int64_t vi = f.v[k].v - 1;
        if (vi < 0 || (uint64_t)vi >= nv) invalid("vertex index out of range");
        for (int c = 0; c < 3; c++) vo[k][c] = (double)(float)o->v[vi * 3 + c];
        if (!without_uvs) {
          const int64_t ti = f.v[k].vt - 1;
          if (ti < 0 || (uint64_t)ti >= nt) invalid("texture coordinate index out of range");
          t.uv[2 * k] = (double)(float)o->vt[ti * 2];
          t.uv[2 * k + 1] = (double)(float)o->vt[ti * 2 + 1];
        }
      }
    }
    return IZPI_OK;
  });
}

}  // extern "C"
