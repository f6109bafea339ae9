// rt_obj.cpp — mesh ingestion on the host: the OBJ
// reader of src/loaders/obj.nim:87-126 (and objconv.nim's copy of it) and
// objconv's .geom writer (objconv.nim:139-153), native so that a
// million-face OBJ loads in a fraction of a second.
//
// Reference semantics restated (obj.nim):
//  * lines split on whitespace (splitWhitespace); only tokens "v" and "f"
//    at the start of a line count ("vn", "vt", "g", "#" ... are skipped);
//  * "v x y z": parseFloat of tokens 1..3; a token that is not entirely a
//    float leaves its coordinate 0 (the `var x: float` default, toVertex);
//  * "f a b c": parseInt(token) - 1 for tokens 1..3 (a 4th vertex is
//    ignored); a token that is not entirely an integer — e.g. "1//2", as in
//    cube-normals.obj — leaves index 0 (toFaceIdx). RT_OBJ_SLASH_INDICES
//    takes the integer before the first '/' instead (the OBJ convention);
//  * a "v" / "f" line with fewer than 4 tokens raises IndexError in Nim:
//    RT_E_IO here.
// objconv(bunny.obj) through these two functions reproduces the reference's
// own test/bunny.geom byte for byte (tests/test_loaders.py).
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rtmi.h"
#include "rt_common.h"

namespace {

bool is_space(char c) { return c == ' ' || c == '\t' || c == '\v' || c == '\r' || c == '\n' || c == '\f'; }

// Nim parseFloat / parseInt: the whole token must parse, else the default 0
double parse_float(const std::string& t) {
  if (t.empty()) return 0.0;
  errno = 0;
  char* end = nullptr;
  const double v = std::strtod(t.c_str(), &end);
  return (end == t.c_str() + t.size()) ? v : 0.0;
}

int64_t parse_index(const std::string& tok, bool slash) {
  std::string t = tok;
  if (slash) {
    const size_t k = t.find('/');
    if (k != std::string::npos) t.resize(k);
  }
  if (t.empty()) return 0;
  errno = 0;
  char* end = nullptr;
  const long long v = std::strtoll(t.c_str(), &end, 10);
  if (end != t.c_str() + t.size() || errno == ERANGE) return 0;
  return (int64_t)v - 1;
}

struct ObjData {
  std::vector<double> v;
  std::vector<int32_t> f;
};

int parse_obj(const char* path, uint32_t flags, bool fill, int64_t* nv, int64_t* nf, ObjData* out) {
  FILE* fp = std::fopen(path, "rb");
  if (!fp) return rtmi_fail_msg(RT_E_IO, (std::string("cannot open ") + path).c_str());
  std::string text;
  char buf[1 << 16];
  size_t got;
  while ((got = std::fread(buf, 1, sizeof buf, fp)) > 0) text.append(buf, got);
  std::fclose(fp);
  const bool slash = (flags & RT_OBJ_SLASH_INDICES) != 0;
  int64_t cv = 0, cf = 0, line_no = 0;
  std::vector<std::string> tok;
  size_t i = 0;
  while (i < text.size()) {
    size_t e = text.find('\n', i);
    if (e == std::string::npos) e = text.size();
    ++line_no;
    tok.clear();
    size_t k = i;
    while (k < e && tok.size() < 4) {  // tokens 0..3 are all either reader looks at
      while (k < e && is_space(text[k])) ++k;
      const size_t b = k;
      while (k < e && !is_space(text[k])) ++k;
      if (k > b) tok.emplace_back(text, b, k - b);
    }
    i = e + 1;
    if (tok.empty()) continue;
    const bool is_v = tok[0] == "v", is_f = tok[0] == "f";
    if (!is_v && !is_f) continue;
    if (tok.size() < 4) {
      char msg[256];
      std::snprintf(msg, sizeof msg, "%s:%lld: '%s' line with fewer than 3 values", path, (long long)line_no,
                    tok[0].c_str());
      return rtmi_fail_msg(RT_E_IO, msg);
    }
    if (is_v) {
      ++cv;
      if (fill)
        for (int a = 1; a <= 3; ++a) out->v.push_back(parse_float(tok[(size_t)a]));
    } else {
      ++cf;
      if (fill)
        for (int a = 1; a <= 3; ++a) {
          const int64_t x = parse_index(tok[(size_t)a], slash);
          if (x < INT32_MIN || x > INT32_MAX) {
            char msg[256];
            std::snprintf(msg, sizeof msg, "%s:%lld: face index out of int32 range", path, (long long)line_no);
            return rtmi_fail_msg(RT_E_IO, msg);
          }
          out->f.push_back((int32_t)x);
        }
    }
  }
  *nv = cv;
  *nf = cf;
  return RT_OK;
}

}  // namespace

extern "C" {

int rt_load_obj(const char* path, uint32_t flags, int64_t* num_vertices, double* vertices, int64_t* num_faces,
                int32_t* faces) {
  if (!path || !num_vertices || !num_faces) return rtmi_fail_msg(RT_E_INVALID, "null argument");
  if (flags & ~(uint32_t)RT_OBJ_SLASH_INDICES) return rtmi_fail_msg(RT_E_INVALID, "unknown flags");
  const bool fill = vertices || faces;
  if (fill && (!vertices || !faces)) return rtmi_fail_msg(RT_E_INVALID, "pass both output buffers or neither");
  ObjData d;
  int64_t nv = 0, nf = 0;
  const int rc = parse_obj(path, flags, fill, &nv, &nf, &d);
  if (rc) return rc;
  if (fill) {
    if (*num_vertices < nv || *num_faces < nf) return rtmi_fail_msg(RT_E_INVALID, "output buffers too small");
    if (!d.v.empty()) std::memcpy(vertices, d.v.data(), d.v.size() * sizeof(double));
    if (!d.f.empty()) std::memcpy(faces, d.f.data(), d.f.size() * sizeof(int32_t));
  }
  *num_vertices = nv;
  *num_faces = nf;
  return RT_OK;
}

int rt_write_geom(const char* path, const double* vertices, int64_t num_vertices, const int32_t* faces,
                  int64_t num_faces) {
  if (!path || (num_faces > 0 && (!vertices || !faces)) || num_vertices < 0 || num_faces < 0)
    return rtmi_fail_msg(RT_E_INVALID, "null or negative argument");
  if (num_faces > INT32_MAX) return rtmi_fail_msg(RT_E_INVALID, "too many faces for a .geom file");
  for (int64_t k = 0; k < num_faces * 3; ++k)
    if (faces[k] < 0 || faces[k] >= num_vertices) return rtmi_fail_msg(RT_E_INVALID, "face index out of range");
  // objconv.nim writeGeom: int32 face count, then per face its three
  // vertices as float32 x, y, z (little-endian, as written on x86)
  std::vector<float> soup((size_t)num_faces * 9);
  for (int64_t t = 0; t < num_faces; ++t)
    for (int k = 0; k < 3; ++k)
      for (int a = 0; a < 3; ++a)
        soup[(size_t)(9 * t + 3 * k + a)] = (float)vertices[3 * (size_t)faces[3 * t + k] + (size_t)a];
  FILE* fp = std::fopen(path, "wb");
  if (!fp) return rtmi_fail_msg(RT_E_IO, (std::string("cannot create ") + path).c_str());
  const int32_t n = (int32_t)num_faces;
  const bool ok = std::fwrite(&n, 4, 1, fp) == 1 &&
                  (soup.empty() || std::fwrite(soup.data(), sizeof(float), soup.size(), fp) == soup.size());
  const bool closed = std::fclose(fp) == 0;
  if (!ok || !closed) return rtmi_fail_msg(RT_E_IO, (std::string("write failed: ") + path).c_str());
  return RT_OK;
}

}  // extern "C"
