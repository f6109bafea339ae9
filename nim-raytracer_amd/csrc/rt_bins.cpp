// rt_bins.cpp — host builders of the float32 kernel's pixel lists and light
// grids (rt_bins.h). float64 throughout; every bound errs on the side of
// listing a face.
#include "rt_bins.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <thread>
#include <unordered_map>

namespace rtmi {

namespace {

// glm column-major: m[c*4 + r]
inline void xform_point(const double m[16], const double p[3], double out[3]) {
  for (int r = 0; r < 3; ++r) out[r] = m[0 * 4 + r] * p[0] + m[1 * 4 + r] * p[1] + m[2 * 4 + r] * p[2] + m[3 * 4 + r];
}
inline void xform_dir(const double m[16], const double d[3], double out[3]) {
  for (int r = 0; r < 3; ++r) out[r] = m[0 * 4 + r] * d[0] + m[1 * 4 + r] * d[1] + m[2 * 4 + r] * d[2];
}
inline double dot3(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
inline void cross3(const double a[3], const double b[3], double o[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
inline double norm3(const double a[3]) { return std::sqrt(dot3(a, a)); }

// Frobenius norm of the 3x3 part: an upper bound of the spectral norm.
double frob3(const double m[16]) {
  double s = 0.0;
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) s += m[c * 4 + r] * m[c * 4 + r];
  return std::sqrt(s);
}

bool invert4(const double m[16], double inv[16]) {
  // Gauss-Jordan with partial pivoting on a row-major copy
  double a[4][8];
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) {
      a[r][c] = m[c * 4 + r];
      a[r][4 + c] = r == c ? 1.0 : 0.0;
    }
  for (int c = 0; c < 4; ++c) {
    int piv = c;
    for (int r = c + 1; r < 4; ++r)
      if (std::fabs(a[r][c]) > std::fabs(a[piv][c])) piv = r;
    if (a[piv][c] == 0.0) return false;
    if (piv != c)
      for (int k = 0; k < 8; ++k) std::swap(a[c][k], a[piv][k]);
    const double d = a[c][c];
    for (int k = 0; k < 8; ++k) a[c][k] /= d;
    for (int r = 0; r < 4; ++r) {
      if (r == c) continue;
      const double f = a[r][c];
      if (f != 0.0)
        for (int k = 0; k < 8; ++k) a[r][k] -= f * a[c][k];
    }
  }
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) inv[c * 4 + r] = a[r][4 + c];
  return true;
}

// The single-sided test rejects det < 1e-6 (geom.nim:306). det is computed
// in float32 from the object-space direction rd and nn = -(e1 x e2); a face
// is left out of a family's bins only when det stays below 1e-6 even with a
// float32 error of 1e-6 * |rd| * |nn| (generous: the test's own rounding is
// ~1e-7 of that).
inline bool never_passes(double det_upper, double rd_max, double nlen) {
  return det_upper + 1e-6 * rd_max * nlen < 1e-6;
}

// Separating-axis test of a 2D triangle against the box [x0, x1] x [y0, y1]
// (the box axes are the caller's bounding-rectangle loop): false only when
// one triangle edge has all four box corners strictly outside it.
// Area of the 2D triangle q[0..5] (x, y pairs) inside the box [x0, x1] x
// [y0, y1]: Sutherland-Hodgman against the four edges, then the shoelace.
inline double clipped_area(const double* q, double x0, double y0, double x1, double y1) {
  double a[16][2], b[16][2];
  int n = 3;
  for (int k = 0; k < 3; ++k) {
    a[k][0] = q[2 * k];
    a[k][1] = q[2 * k + 1];
  }
  // edge e: keep points with s * p[axis] <= s * lim
  const int axis[4] = {0, 0, 1, 1};
  const double lim[4] = {x0, x1, y0, y1}, sgn[4] = {-1.0, 1.0, -1.0, 1.0};
  for (int ei = 0; ei < 4 && n > 0; ++ei) {
    const int ax = axis[ei];
    int m = 0;
    for (int k = 0; k < n; ++k) {
      const double* P = a[k];
      const double* Q = a[(k + 1) % n];
      const double dp = sgn[ei] * (P[ax] - lim[ei]), dq = sgn[ei] * (Q[ax] - lim[ei]);
      if (dp <= 0.0) {
        b[m][0] = P[0];
        b[m][1] = P[1];
        ++m;
      }
      if ((dp < 0.0 && dq > 0.0) || (dp > 0.0 && dq < 0.0)) {
        const double t = dp / (dp - dq);
        b[m][0] = P[0] + t * (Q[0] - P[0]);
        b[m][1] = P[1] + t * (Q[1] - P[1]);
        ++m;
      }
    }
    n = m;
    for (int k = 0; k < n; ++k) {
      a[k][0] = b[k][0];
      a[k][1] = b[k][1];
    }
  }
  double area = 0.0;
  for (int k = 0; k < n; ++k) {
    const double* P = a[k];
    const double* Q = a[(k + 1) % n];
    area += P[0] * Q[1] - Q[0] * P[1];
  }
  return 0.5 * std::fabs(area);
}

inline bool tri_meets_box(const double* q, double x0, double y0, double x1, double y1) {
  const double area = (q[2] - q[0]) * (q[5] - q[1]) - (q[3] - q[1]) * (q[4] - q[0]);
  if (!(area != 0.0)) return true;  // degenerate (or NaN): keep
  const double sg = area > 0.0 ? 1.0 : -1.0;
  const double cx[4] = {x0, x1, x0, x1}, cy[4] = {y0, y0, y1, y1};
  for (int k = 0; k < 3; ++k) {
    const double ax = q[2 * k], ay = q[2 * k + 1];
    const double bx = q[2 * ((k + 1) % 3)], by = q[2 * ((k + 1) % 3) + 1];
    double best = -INFINITY;
    for (int c = 0; c < 4; ++c) best = std::max(best, sg * ((bx - ax) * (cy[c] - ay) - (by - ay) * (cx[c] - ax)));
    if (best < 0.0) return false;
  }
  return true;
}

// Two-pass bucket fill: count[k] entries per bin -> off (prefix) -> ent.
template <class Emit>
bool fill_bins(size_t nbins, size_t ntri, Emit emit, std::vector<int32_t>& off, std::vector<int32_t>& ent,
               const char** why) {
  std::vector<int64_t> cnt(nbins + 1, 0);
  for (size_t i = 0; i < ntri; ++i) emit(i, [&](size_t b, int32_t) { ++cnt[b + 1]; });
  for (size_t b = 0; b < nbins; ++b) cnt[b + 1] += cnt[b];
  if (cnt[nbins] + kBinPad > std::numeric_limits<int32_t>::max()) {
    *why = "too many bin entries";
    return false;
  }
  off.assign(cnt.begin(), cnt.end());
  ent.assign((size_t)cnt[nbins] + kBinPad, 0);
  std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
  for (size_t i = 0; i < ntri; ++i) emit(i, [&](size_t b, int32_t rec) { ent[(size_t)pos[b]++] = rec; });
  // padding repeats the last record: a read-ahead never leaves the tree
  for (int k = 0; k < kBinPad; ++k) ent[(size_t)cnt[nbins] + k] = cnt[nbins] > 0 ? ent[(size_t)cnt[nbins] - 1] : 0;
  return true;
}

}  // namespace

bool pixel_camera(const double o2w[16], const double w2o[16], const double c2w[16], double fov_deg, int width,
                  int height, bg::PixCam* out) {
  if (!invert4(c2w, out->w2c)) return false;
  std::memcpy(out->o2w, o2w, sizeof out->o2w);
  // camera constants of the float32 kernel (rtmi.cpp fill_fast): a camera-space
  // direction (cx, cy, -1) is the sample at px = w/2 + cx/a, py = h/2 - cy/c
  const double f = std::tan(fov_deg * (3.14159265358979323846 / 180.0) / 2);
  const double r = (double)width / (double)height;
  out->cam_a = 2.0 * r * f / (double)width;
  out->cam_c = 2.0 * f / (double)height;
  const double cw[3] = {c2w[12], c2w[13], c2w[14]};
  xform_point(w2o, cw, out->co);  // camera origin in object space
  // |rd| of a unit world direction lies in [1/|o2w|, |w2o|]
  out->rd_max = frob3(w2o);
  out->rd_min = 1.0 / frob3(o2w);
  out->margin = kPixelMargin;
  out->width = width;
  out->height = height;
  return true;
}

bool skip_camera(const std::vector<SkipPlane>& planes, const double mesh_w2o[16], const double c2w[16],
                 double fov_deg, int width, int height, double bias, bg::SkipCam* cam,
                 std::vector<bg::SkipPlaneC>* pc) {
  std::memcpy(cam->c2w, c2w, sizeof cam->c2w);
  std::memcpy(cam->mesh_w2o, mesh_w2o, sizeof cam->mesh_w2o);
  for (int k = 0; k < 3; ++k) cam->cw[k] = c2w[12 + k];
  const double f = std::tan(fov_deg * (3.14159265358979323846 / 180.0) / 2);
  const double r = (double)width / (double)height;
  cam->cam_a = 2.0 * r * f / (double)width;
  cam->cam_c = 2.0 * f / (double)height;
  cam->margin = kPixelMargin;
  cam->bias = bias;
  cam->width = width;
  cam->height = height;
  pc->assign(planes.size(), bg::SkipPlaneC{});
  for (size_t k = 0; k < planes.size(); ++k) {
    double o[3];
    xform_point(planes[k].w2o, cam->cw, o);
    bg::SkipPlaneC& P = (*pc)[k];
    P.oy = o[1];
    for (int c = 0; c < 3; ++c) {
      P.row[c] = planes[k].w2o[c * 4 + 1];
      P.n[c] = planes[k].o2w[1 * 4 + c];
    }
    P.tol = 1e-5 * frob3(planes[k].w2o);
    if (!(std::fabs(o[1]) > 1e-9)) return false;  // the camera lies on a plane: no pixel qualifies
  }
  return true;
}

bool build_pixel_bins(const std::vector<BinTri>& tris, const double o2w[16], const double w2o[16],
                      const double c2w[16], double fov_deg, int width, int height, PixelBinsHost* out,
                      const char** why) {
  *why = "";
  if (width <= 0 || height <= 0) {
    *why = "empty image";
    return false;
  }
  bg::PixCam pc;
  if (!pixel_camera(o2w, w2o, c2w, fov_deg, width, height, &pc)) {
    *why = "singular camera";
    return false;
  }
  const double margin = kPixelMargin;
  // per face: pixel rectangle (or empty) and projected vertices
  // (rt_bins_geom.h face_pixel_rect, shared with the per-frame device builder)
  std::vector<int32_t> rect(tris.size() * 4, -1);
  std::vector<double> proj(tris.size() * 6, 0.0);
  for (size_t i = 0; i < tris.size(); ++i) {
    if (!bg::face_pixel_rect(pc, tris[i].v, &proj[6 * i], &rect[4 * i])) {
      *why = "a mesh vertex lies at or behind the camera plane";
      return false;
    }
  }
  auto emit = [&](size_t i, auto&& put) {
    if (rect[4 * i] < 0) return;
    const double* q = &proj[6 * i];
    for (int32_t y = rect[4 * i + 2]; y <= rect[4 * i + 3]; ++y)
      for (int32_t x = rect[4 * i + 0]; x <= rect[4 * i + 1]; ++x)
        if (bg::tri_meets_box(q, x - margin, y - margin, x + 1 + margin, y + 1 + margin))
          put((size_t)y * (size_t)width + (size_t)x, tris[i].rec);
  };
  return fill_bins((size_t)width * (size_t)height, tris.size(), emit, out->off, out->ent, why);
}

bool build_light_grid(const std::vector<BinTri>& tris, const double w2o[16], const double dir[3],
                      LightGridHost* out, const char** why) {
  *why = "";
  out->g = LightGrid{};
  const double sd[3] = {-dir[0], -dir[1], -dir[2]};
  double rd[3];
  xform_dir(w2o, sd, rd);  // object-space shadow direction (the kernel's rd, up to float32 rounding)
  const double rlen = norm3(rd);
  if (!(rlen > 0.0) || !std::isfinite(rlen)) {
    *why = "degenerate light direction";
    return false;
  }
  const double u[3] = {rd[0] / rlen, rd[1] / rlen, rd[2] / rlen};
  // basis orthogonal to the shadow direction
  const int ax = std::fabs(u[0]) <= std::fabs(u[1]) && std::fabs(u[0]) <= std::fabs(u[2]) ? 0
                 : std::fabs(u[1]) <= std::fabs(u[2])                                 ? 1
                                                                                      : 2;
  double a[3] = {0, 0, 0};
  a[ax] = 1.0;
  double e1[3], e2[3];
  cross3(a, u, e1);
  const double l1 = norm3(e1);
  for (double& x : e1) x /= l1;
  cross3(u, e1, e2);
  double scale = 1.0;
  for (const BinTri& t : tris)
    for (int v = 0; v < 3; ++v)
      for (int k = 0; k < 3; ++k) scale = std::max(scale, std::fabs(t.v[v][k]));
  const double delta = 1e-5 * scale;
  std::vector<double> box(tris.size() * 4, NAN), proj(tris.size() * 6, 0.0);
  double umin = INFINITY, umax = -INFINITY, vmin = INFINITY, vmax = -INFINITY;
  size_t kept = 0;
  for (size_t i = 0; i < tris.size(); ++i) {
    const BinTri& t = tris[i];
    double f1[3], f2[3], c[3], nn[3];
    for (int k = 0; k < 3; ++k) {
      f1[k] = t.v[1][k] - t.v[0][k];
      f2[k] = t.v[2][k] - t.v[0][k];
    }
    cross3(f1, f2, c);
    for (int k = 0; k < 3; ++k) nn[k] = -c[k];
    if (never_passes(dot3(rd, nn), rlen, norm3(nn))) continue;  // faces away from the light
    double bu0 = INFINITY, bu1 = -INFINITY, bv0 = INFINITY, bv1 = -INFINITY;
    for (int v = 0; v < 3; ++v) {
      const double pu = dot3(t.v[v], e1), pv = dot3(t.v[v], e2);
      proj[6 * i + 2 * v] = pu;
      proj[6 * i + 2 * v + 1] = pv;
      bu0 = std::min(bu0, pu);
      bu1 = std::max(bu1, pu);
      bv0 = std::min(bv0, pv);
      bv1 = std::max(bv1, pv);
    }
    box[4 * i + 0] = bu0 - delta;
    box[4 * i + 1] = bu1 + delta;
    box[4 * i + 2] = bv0 - delta;
    box[4 * i + 3] = bv1 + delta;
    umin = std::min(umin, box[4 * i + 0]);
    umax = std::max(umax, box[4 * i + 1]);
    vmin = std::min(vmin, box[4 * i + 2]);
    vmax = std::max(vmax, box[4 * i + 3]);
    ++kept;
  }
  LightGrid& g = out->g;
  for (int k = 0; k < 3; ++k) {
    g.e1[k] = (float)e1[k];
    g.e2[k] = (float)e2[k];
  }
  g.rmax = (float)(100.0 * scale);
  if (kept == 0) {  // nothing faces the light: every lane misses (an empty 1x1 grid)
    g.u0 = g.v0 = 0.0f;
    g.inv_h = 1.0f;
    g.gu = g.gv = 1;
    out->off.assign(2, 0);
    out->ent.assign(kBinPad, tris.empty() ? 0 : tris[0].rec);
    return true;
  }
  // about 2 cells per listed face (RTMI_GRID_DENSITY), square cells, at most
  // 4096 per side. Coarse cells measured best on C3: density 1 / 2 / 4 / 8 /
  // 16 / 32 -> 4.91 / 4.89 / 4.92 / 4.96 / 5.09 / 5.76 ms (fewer distinct
  // cells per wave, fewer lanes left to the BVH, more record reuse)
  static const double density = [] {
    const char* e = rtmi::diag_env("RTMI_GRID_DENSITY");
    const double v = e ? std::atof(e) : 2.0;
    return v > 0.0 ? v : 2.0;
  }();
  const double du = std::max(umax - umin, 1e-30), dv = std::max(vmax - vmin, 1e-30);
  double h = std::sqrt(du * dv / (density * (double)kept));
  h = std::max(h, std::max(du, dv) / 4096.0);
  const int gu = std::max(1, std::min(4096, (int)std::ceil(du / h)));
  const int gv = std::max(1, std::min(4096, (int)std::ceil(dv / h)));
  // the float32 origin / cell size the kernel uses, so host and device agree on
  // cell edges up to float32 rounding (covered by delta)
  g.u0 = (float)umin;
  g.v0 = (float)vmin;
  g.inv_h = (float)(1.0 / h);
  g.gu = gu;
  g.gv = gv;
  const double ih = (double)g.inv_h;
  auto emit = [&](size_t i, auto&& put) {
    if (std::isnan(box[4 * i])) return;
    const int c0 = std::max(0, (int)std::floor((box[4 * i + 0] - (double)g.u0) * ih));
    const int c1 = std::min(gu - 1, (int)std::floor((box[4 * i + 1] - (double)g.u0) * ih));
    const int r0 = std::max(0, (int)std::floor((box[4 * i + 2] - (double)g.v0) * ih));
    const int r1 = std::min(gv - 1, (int)std::floor((box[4 * i + 3] - (double)g.v0) * ih));
    const double* q = &proj[6 * i];
    for (int r = r0; r <= r1; ++r)
      for (int c = c0; c <= c1; ++c) {
        const double cu0 = (double)g.u0 + c / ih, cv0 = (double)g.v0 + r / ih;
        if (tri_meets_box(q, cu0 - delta, cv0 - delta, cu0 + 1.0 / ih + delta, cv0 + 1.0 / ih + delta))
          put((size_t)r * (size_t)gu + (size_t)c, tris[i].rec);
      }
  };
  if (!fill_bins((size_t)gu * (size_t)gv, tris.size(), emit, out->off, out->ent, why)) return false;
  out->box = box;
  out->rec0 = tris.empty() ? 0 : tris[0].rec;
  // each cell's faces ordered by the share of the cell their projection
  // covers, largest first: a shadow ray in the umbra meets the covering face
  // first, and the kernels' early exit (checked after a cell's first face)
  // retires it after one test. Order never changes a result (any order
  // finds the same closest t; an early exit only needs some hit <= stop).
  std::unordered_map<int32_t, int32_t> face_of;
  face_of.reserve(tris.size());
  for (size_t i = 0; i < tris.size(); ++i)
    if (!std::isnan(box[4 * i])) face_of.emplace(tris[i].rec, (int32_t)i);
  const double hc = 1.0 / ih;
  std::vector<std::pair<double, int32_t>> row;
  for (int r = 0; r < gv; ++r)
    for (int c = 0; c < gu; ++c) {
      const size_t cell = (size_t)r * (size_t)gu + (size_t)c;
      const int32_t b = out->off[cell], e = out->off[cell + 1];
      if (e - b < 2) continue;
      const double cu0 = (double)g.u0 + c * hc, cv0 = (double)g.v0 + r * hc;
      row.clear();
      for (int32_t k = b; k < e; ++k) {
        const int32_t rec = out->ent[(size_t)k];
        const auto it = face_of.find(rec);
        const double cov = it == face_of.end() ? 0.0 : clipped_area(&proj[6 * (size_t)it->second], cu0, cv0, cu0 + hc, cv0 + hc);
        row.emplace_back(-cov, rec);
      }
      std::stable_sort(row.begin(), row.end(),
                       [](const std::pair<double, int32_t>& x, const std::pair<double, int32_t>& y) { return x.first < y.first; });
      for (int32_t k = b; k < e; ++k) out->ent[(size_t)k] = row[(size_t)(k - b)].second;
    }
  return true;
}

void skip_grid(const GridOcc& go, bg::SkipGrid* out) {
  const LightGrid& g = go.g;
  for (int k = 0; k < 3; ++k) {
    out->e1[k] = g.e1[k];
    out->e2[k] = g.e2[k];
  }
  out->u0 = g.u0;
  out->v0 = g.v0;
  out->inv_h = g.inv_h;
  out->gu = g.gu;
  out->gv = g.gv;
  out->sat = go.sat.empty() ? nullptr : go.sat.data();
}

void grid_occupancy(const LightGridHost& lg, GridOcc* out) {
  out->g = lg.g;
  out->sat.clear();
  const int gu = lg.g.gu, gv = lg.g.gv;
  if (gu <= 0 || gv <= 0 || (int64_t)lg.off.size() < (int64_t)gu * gv + 1) {
    out->g.gu = 0;
    return;
  }
  out->sat.assign((size_t)(gu + 1) * (size_t)(gv + 1), 0);
  for (int v = 0; v < gv; ++v) {
    int32_t row = 0;
    for (int u = 0; u < gu; ++u) {
      const size_t c = (size_t)v * gu + u;
      row += lg.off[c + 1] > lg.off[c] ? 1 : 0;
      out->sat[(size_t)(v + 1) * (gu + 1) + u + 1] = out->sat[(size_t)v * (gu + 1) + u + 1] + row;
    }
  }
}

bool build_shadow_skips(const std::vector<int32_t>& pix_off, const std::vector<SkipPlane>& planes,
                        const double mesh_w2o[16], const std::vector<GridOcc>& grids, const double c2w[16],
                        double fov_deg, int width, int height, double bias, std::vector<uint32_t>* out,
                        const char** why, std::vector<int32_t>* sl, std::vector<int32_t>* sl_ent, int sl_nl) {
  *why = "";
  const size_t npx = (size_t)width * (size_t)height;
  if (width <= 0 || height <= 0 || pix_off.size() != npx + 1) {
    *why = "pixel lists of another size";
    return false;
  }
  out->assign((npx + 3) / 4, 0u);
  const int nl = std::min<int>(8, (int)grids.size());
  if (sl) {
    sl->assign(npx * (size_t)sl_nl * 2, -1);
    sl_ent->clear();
  }
  unsigned have = 0;
  for (int l = 0; l < nl; ++l) have |= grids[(size_t)l].g.gu > 0 ? 1u << l : 0u;
  if (have == 0) return true;
  if (!sl || sl_nl <= 0) {  // the bits alone: rt_bins_geom.h pixel_skip_bits, as the device builder forms them
    bg::SkipCam cam;
    std::vector<bg::SkipPlaneC> pcs;
    if (!skip_camera(planes, mesh_w2o, c2w, fov_deg, width, height, bias, &cam, &pcs)) {
      *why = "the camera lies on a plane";
      return true;  // no pixel qualifies
    }
    std::vector<bg::SkipGrid> sg((size_t)nl);
    for (int l = 0; l < nl; ++l) skip_grid(grids[(size_t)l], &sg[(size_t)l]);
    std::vector<uint8_t> bytes(npx, 0);
    auto rows = [&](int64_t ya, int64_t yb) {
      for (int64_t y = ya; y < yb; ++y)
        for (int x = 0; x < width; ++x) {
          const size_t pix = (size_t)y * width + x;
          if (pix_off[pix + 1] != pix_off[pix]) continue;  // camera rays may hit the mesh
          bytes[pix] = (uint8_t)bg::pixel_skip_bits(cam, pcs.data(), (int)pcs.size(), sg.data(), nl, have, x, (int)y);
        }
    };
    const int nt = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (nt == 1 || npx < 65536) {
      rows(0, height);
    } else {
      std::vector<std::thread> th;
      const int chunk = (height + nt - 1) / nt;
      for (int t = 0; t < nt; ++t) {
        const int ya = t * chunk, yb = std::min(height, ya + chunk);
        if (ya < yb) th.emplace_back(rows, ya, yb);
      }
      for (auto& t : th) t.join();
    }
    for (size_t pix = 0; pix < npx; ++pix) (*out)[pix >> 2] |= (uint32_t)bytes[pix] << (8 * (pix & 3));
    return true;
  }
  // the kernel's camera constants (as in build_pixel_bins); a corner ray of
  // pixel (x, y) passes through (x +- margin, y +- margin)
  const double f = std::tan(fov_deg * (3.14159265358979323846 / 180.0) / 2);
  const double r = (double)width / (double)height;
  const double cam_a = 2.0 * r * f / (double)width, cam_c = 2.0 * f / (double)height;
  const double margin = kPixelMargin;
  const double cw[3] = {c2w[12], c2w[13], c2w[14]};
  struct PlaneC {
    double oy;        // camera origin's object-space y
    double row[3];    // object-space y of a world direction: row . d
    double n[3];      // world normal (object_to_world * (0, 1, 0), as the kernel's N)
    double tol;       // float32 error allowance of row . d
  };
  std::vector<PlaneC> pc(planes.size());
  for (size_t k = 0; k < planes.size(); ++k) {
    double o[3];
    xform_point(planes[k].w2o, cw, o);
    pc[k].oy = o[1];
    for (int c = 0; c < 3; ++c) {
      pc[k].row[c] = planes[k].w2o[c * 4 + 1];
      pc[k].n[c] = planes[k].o2w[1 * 4 + c];
    }
    pc[k].tol = 1e-5 * frob3(planes[k].w2o);
    if (!(std::fabs(o[1]) > 1e-9)) {
      *why = "the camera lies on a plane";
      return true;  // no pixel qualifies
    }
  }
  // rows in parallel (host threads), one byte per pixel, packed below; the
  // shadow lists per thread, merged after
  std::vector<uint8_t> bytes(npx, 0);
  struct ListPart {
    std::vector<int32_t> ent;
    std::vector<std::array<int64_t, 3>> at;  // (pix * sl_nl + l, start in ent, count)
  };
  const bool want_lists = sl != nullptr && sl_nl > 0;
  auto rows = [&](int ya, int yb, ListPart* part) {
  std::vector<std::pair<double, int32_t>> cand[8];
  // per light, the last (pixel + 1) that listed a face: duplicates from
  // neighbouring cells are dropped as they are gathered (no sort / unique)
  std::vector<uint32_t> seen[8];
  for (int y = ya; y < yb; ++y) {
    for (int x = 0; x < width; ++x) {
      const size_t pix = (size_t)y * width + x;
      if (pix_off[pix + 1] != pix_off[pix]) continue;  // camera rays may hit the mesh
      double dw[4][3];
      for (int c = 0; c < 4; ++c) {
        const double px = (c & 1) ? x + 1 + margin : x - margin, py = (c & 2) ? y + 1 + margin : y - margin;
        const double dc[3] = {(px - 0.5 * width) * cam_a, (0.5 * height - py) * cam_c, -1.0};
        xform_dir(c2w, dc, dw[c]);
        const double len = norm3(dw[c]);
        for (int k = 0; k < 3; ++k) dw[c][k] /= len;
      }
      unsigned bits = have, bad = 0u;
      bool qualified = true;
      for (int l = 0; l < nl; ++l) cand[l].clear();
      for (size_t k = 0; k < planes.size() && bits; ++k) {
        const PlaneC& P = pc[k];
        int hit = 0, miss = 0;
        double t[4];
        for (int c = 0; c < 4; ++c) {
          const double dy = dot3(P.row, dw[c]);
          // the kernel counts a plane hit at t = -oy / dy >= 0 with |dy| > 1e-6
          const double s = P.oy > 0.0 ? -dy : dy;  // > 0: towards the plane
          if (s > P.tol + 1e-6) {
            ++hit;
            t[c] = -P.oy / dy;
          } else if (s < -P.tol) {
            ++miss;
          }
        }
        if (miss == 4) continue;  // no ray of the pixel reaches this plane
        if (hit != 4) {           // a horizon inside the pixel: unbounded footprint
          bits = 0;
          qualified = false;
          break;
        }
        for (int l = 0; l < nl; ++l) {
          if (!(bits >> l & 1u) && !want_lists) continue;
          const LightGrid& g = grids[(size_t)l].g;
          if (g.gu <= 0) continue;
          const double e1[3] = {g.e1[0], g.e1[1], g.e1[2]}, e2[3] = {g.e2[0], g.e2[1], g.e2[2]};
          double umin = INFINITY, umax = -INFINITY, vmin = INFINITY, vmax = -INFINITY, qmax = 0.0;
          for (int c = 0; c < 4; ++c) {
            // shadow-ray origin: hit + N * bias (renderer.nim:94-101), in mesh space
            const double so[3] = {cw[0] + dw[c][0] * t[c] + P.n[0] * bias, cw[1] + dw[c][1] * t[c] + P.n[1] * bias,
                                  cw[2] + dw[c][2] * t[c] + P.n[2] * bias};
            double q[3];
            xform_point(mesh_w2o, so, q);
            qmax = std::max(qmax, std::max(std::fabs(q[0]), std::max(std::fabs(q[1]), std::fabs(q[2]))));
            const double u = dot3(q, e1), v = dot3(q, e2);
            umin = std::min(umin, u);
            umax = std::max(umax, u);
            vmin = std::min(vmin, v);
            vmax = std::max(vmax, v);
          }
          // the footprint as rt_bins_geom.h rect_skip_bits forms it (float32
          // margins far inside 1e-4 of the magnitudes; no extra cell)
          const double mw = 1e-4 * (1.0 + qmax) + 1e-4 * std::fabs(bias);
          const double ih = g.inv_h;
          const double fu0 = (umin - mw - g.u0) * ih - RTMI_SKIP_CELL_PAD, fu1 = (umax + mw - g.u0) * ih + RTMI_SKIP_CELL_PAD;
          const double fv0 = (vmin - mw - g.v0) * ih - RTMI_SKIP_CELL_PAD, fv1 = (vmax + mw - g.v0) * ih + RTMI_SKIP_CELL_PAD;
          if (!(fu1 >= 0.0 && fv1 >= 0.0 && fu0 < g.gu && fv0 < g.gv)) continue;  // off the grid
          if (!std::isfinite(fu0 + fu1 + fv0 + fv1)) {
            bits &= ~(1u << l);
            bad |= 1u << l;
            continue;
          }
          // a list stands in for the kernel's float32-safe-radius check
          // (origins beyond rmax take the BVH): keep well inside it
          const bool far = !(qmax <= 0.5 * (double)g.rmax);
          const int u0 = (int)std::max(0.0, std::floor(fu0)), u1 = (int)std::min((double)g.gu - 1, std::floor(fu1));
          const int v0 = (int)std::max(0.0, std::floor(fv0)), v1 = (int)std::min((double)g.gv - 1, std::floor(fv1));
          const std::vector<int32_t>& S = grids[(size_t)l].sat;
          const size_t W1 = (size_t)g.gu + 1;
          const int32_t n = S[(size_t)(v1 + 1) * W1 + u1 + 1] - S[(size_t)v0 * W1 + u1 + 1] -
                            S[(size_t)(v1 + 1) * W1 + u0] + S[(size_t)v0 * W1 + u0];
          if (n == 0) continue;
          bits &= ~(1u << l);
          // the shadow list: faces of those cells whose grown projected box
          // meets the footprint grown by mw (a hit face's box must)
          const LightGridHost* L = grids[(size_t)l].lists;
          // a footprint over many cells (towards the horizon) would list more
          // faces than the cells the kernel would search: no list
          const bool wide = (int64_t)(u1 - u0 + 1) * (int64_t)(v1 - v0 + 1) > 36;
          if (!want_lists || l >= sl_nl || !L || far || wide) {
            bad |= 1u << l;
            continue;
          }
          const double ru0 = umin - mw, ru1 = umax + mw, rv0 = vmin - mw, rv1 = vmax + mw;
          std::vector<uint32_t>& sn = seen[l];
          if (sn.size() < L->box.size() / 4) sn.assign(L->box.size() / 4, 0u);
          const uint32_t stamp = (uint32_t)pix + 1u;
          for (int cv = v0; cv <= v1; ++cv)
            for (int cu = u0; cu <= u1; ++cu) {
              const size_t cell = (size_t)cv * (size_t)g.gu + (size_t)cu;
              for (int32_t e = L->off[cell]; e < L->off[cell + 1]; ++e) {
                const int32_t rec = L->ent[(size_t)e];
                const size_t fi = (size_t)((rec - L->rec0) / (int32_t)sizeof(TriFast));
                if (sn[fi] == stamp) continue;
                const double* fb = &L->box[4 * fi];
                const double ou = std::min(fb[1], ru1) - std::max(fb[0], ru0);
                const double ov = std::min(fb[3], rv1) - std::max(fb[2], rv0);
                if (ou >= 0.0 && ov >= 0.0) {
                  sn[fi] = stamp;
                  cand[l].emplace_back(-ou * ov, rec);
                }
              }
            }
          if (cand[l].size() > 4 * (size_t)kShadowListMax) bad |= 1u << l;
        }
      }
      bytes[pix] = (uint8_t)bits;
      if (!want_lists || !qualified) continue;
      for (int l = 0; l < std::min(nl, sl_nl); ++l) {
        if ((bits >> l & 1u) || (bad >> l & 1u) || grids[(size_t)l].g.gu <= 0) continue;
        auto& c = cand[l];  // one entry per face (the stamps), every plane's footprint
        if (c.size() > (size_t)kShadowListMax) continue;
        // the faces covering most of the footprint first (early exit)
        std::stable_sort(c.begin(), c.end(), [](const std::pair<double, int32_t>& a,
                                                const std::pair<double, int32_t>& b) { return a.first < b.first; });
        part->at.push_back({(int64_t)(pix * (size_t)sl_nl + (size_t)l), (int64_t)part->ent.size(), (int64_t)c.size()});
        for (const auto& e : c) part->ent.push_back(e.second);
      }
    }
  }
  };
  const int nt = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<ListPart> parts((size_t)std::max(1, nt));
  if (nt == 1 || npx < 65536) {
    rows(0, height, &parts[0]);
  } else {
    std::vector<std::thread> th;
    const int chunk = (height + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
      const int ya = t * chunk, yb = std::min(height, ya + chunk);
      if (ya < yb) th.emplace_back(rows, ya, yb, &parts[(size_t)t]);
    }
    for (auto& t : th) t.join();
  }
  if (want_lists) {
    for (const ListPart& pt : parts) {
      const int64_t base = (int64_t)sl_ent->size();
      if (base + (int64_t)pt.ent.size() > INT32_MAX) break;
      for (const auto& a : pt.at) {
        (*sl)[2 * (size_t)a[0]] = (int32_t)(base + a[1]);
        (*sl)[2 * (size_t)a[0] + 1] = (int32_t)a[2];
      }
      sl_ent->insert(sl_ent->end(), pt.ent.begin(), pt.ent.end());
    }
    for (int k = 0; k < kBinPad; ++k) sl_ent->push_back(sl_ent->empty() ? 0 : sl_ent->back());  // read-ahead pad
  }
  for (size_t pix = 0; pix < npx; ++pix) (*out)[pix >> 2] |= (uint32_t)bytes[pix] << (8 * (pix & 3));
  return true;
}

}  // namespace rtmi

namespace rtmi {

bool build_object_pixel_masks(const std::vector<ObjBox>& objs, const double c2w[16], double fov_deg, int width,
                              int height, std::vector<unsigned long long>* masks, const char** why) {
  *why = "";
  if (objs.size() > 64 || width <= 0 || height <= 0) {
    *why = "object masks hold at most 64 objects";
    return false;
  }
  double w2c[16];
  if (!invert4(c2w, w2c)) {
    *why = "singular camera";
    return false;
  }
  const double f = std::tan(fov_deg * (3.14159265358979323846 / 180.0) / 2);
  const double r = (double)width / (double)height;
  const double cam_a = 2.0 * r * f / (double)width, cam_c = 2.0 * f / (double)height;
  const double margin = kPixelMargin;
  unsigned long long always = 0;
  std::vector<std::array<int, 4>> rect(objs.size(), std::array<int, 4>{-1, -1, -1, -1});
  for (size_t i = 0; i < objs.size(); ++i) {
    const ObjBox& b = objs[i];
    bool proj = !b.always;
    double xmin = INFINITY, xmax = -INFINITY, ymin = INFINITY, ymax = -INFINITY;
    for (int c = 0; proj && c < 8; ++c) {
      const double pw[3] = {(c & 1) ? b.hi[0] : b.lo[0], (c & 2) ? b.hi[1] : b.lo[1], (c & 4) ? b.hi[2] : b.lo[2]};
      double pc[3];
      xform_point(w2c, pw, pc);
      if (!(pc[2] < -1e-9 * (1.0 + std::fabs(pc[0]) + std::fabs(pc[1])))) {
        proj = false;  // a corner at or behind the camera plane: no bounded projection
        break;
      }
      const double px = 0.5 * width + (pc[0] / -pc[2]) / cam_a;
      const double py = 0.5 * height - (pc[1] / -pc[2]) / cam_c;
      xmin = std::min(xmin, px);
      xmax = std::max(xmax, px);
      ymin = std::min(ymin, py);
      ymax = std::max(ymax, py);
    }
    if (!proj) {
      always |= 1ull << i;
      continue;
    }
    if (!(xmax + margin >= 0.0 && ymax + margin >= 0.0 && xmin - margin < width && ymin - margin < height)) continue;
    rect[i] = {(int)std::max(0.0, std::floor(xmin - margin)), (int)std::min((double)width - 1, std::floor(xmax + margin)),
               (int)std::max(0.0, std::floor(ymin - margin)), (int)std::min((double)height - 1, std::floor(ymax + margin))};
  }
  masks->assign((size_t)width * (size_t)height, always);
  for (size_t i = 0; i < objs.size(); ++i) {
    if (rect[i][0] < 0) continue;
    for (int y = rect[i][2]; y <= rect[i][3]; ++y)
      for (int x = rect[i][0]; x <= rect[i][1]; ++x) (*masks)[(size_t)y * (size_t)width + (size_t)x] |= 1ull << i;
  }
  return true;
}

// Convex hull of 2D points (Andrew's monotone chain), counter-clockwise,
// collinear points dropped.
std::vector<std::array<double, 2>> convex_hull_2d(std::vector<std::array<double, 2>> p) {
  std::sort(p.begin(), p.end());
  p.erase(std::unique(p.begin(), p.end()), p.end());
  if (p.size() < 3) return p;
  auto cross = [](const std::array<double, 2>& o, const std::array<double, 2>& a, const std::array<double, 2>& b) {
    return (a[0] - o[0]) * (b[1] - o[1]) - (a[1] - o[1]) * (b[0] - o[0]);
  };
  std::vector<std::array<double, 2>> h(2 * p.size());
  size_t k = 0;
  for (size_t i = 0; i < p.size(); ++i) {
    while (k >= 2 && cross(h[k - 2], h[k - 1], p[i]) <= 0.0) --k;
    h[k++] = p[i];
  }
  for (size_t i = p.size() - 1, t = k + 1; i-- > 0;) {
    while (k >= t && cross(h[k - 2], h[k - 1], p[i]) <= 0.0) --k;
    h[k++] = p[i];
  }
  h.resize(k - 1);
  return h;
}

// Whether a convex polygon (counter-clockwise) meets the box [u0, u1] x
// [v0, v1]: separating axis test over the box's axes and the polygon's edge
// normals (touching counts as meeting).
bool hull_meets_box(const std::vector<std::array<double, 2>>& h, double u0, double v0, double u1, double v1) {
  double pu0 = INFINITY, pu1 = -INFINITY, pv0 = INFINITY, pv1 = -INFINITY;
  for (const auto& q : h) {
    pu0 = std::min(pu0, q[0]);
    pu1 = std::max(pu1, q[0]);
    pv0 = std::min(pv0, q[1]);
    pv1 = std::max(pv1, q[1]);
  }
  if (pu1 < u0 || pu0 > u1 || pv1 < v0 || pv0 > v1) return false;
  const size_t n = h.size();
  for (size_t i = 0; i < n; ++i) {
    const auto& a = h[i];
    const auto& b = h[(i + 1) % n];
    const double nx = b[1] - a[1], ny = a[0] - b[0];  // outward normal of a CCW edge
    const double lim = nx * a[0] + ny * a[1];
    // the box lies wholly outside this edge when its nearest corner does
    const double m = std::min(std::min(nx * u0 + ny * v0, nx * u1 + ny * v0), std::min(nx * u0 + ny * v1, nx * u1 + ny * v1));
    if (m > lim) return false;
  }
  return true;
}

bool build_object_light_grid(const std::vector<ObjBox>& objs, const double dir[3], ObjGridHost* out,
                             const char** why) {
  *why = "";
  out->g = LightGrid{};
  out->masks.clear();
  out->off_grid = 0;
  if (objs.size() > 64) {
    *why = "object masks hold at most 64 objects";
    return false;
  }
  double u[3] = {-dir[0], -dir[1], -dir[2]};
  const double ul = norm3(u);
  if (!(ul > 0.0) || !std::isfinite(ul)) {
    *why = "degenerate light direction";
    return false;
  }
  for (double& x : u) x /= ul;
  const int ax = std::fabs(u[0]) <= std::fabs(u[1]) && std::fabs(u[0]) <= std::fabs(u[2]) ? 0
                 : std::fabs(u[1]) <= std::fabs(u[2])                                 ? 1
                                                                                      : 2;
  double a[3] = {0, 0, 0};
  a[ax] = 1.0;
  double e1[3], e2[3];
  cross3(a, u, e1);
  const double l1 = norm3(e1);
  for (double& x : e1) x /= l1;
  cross3(u, e1, e2);
  double scale = 1.0;
  for (const ObjBox& b : objs)
    if (!b.always)
      for (int k = 0; k < 3; ++k) scale = std::max(scale, std::max(std::fabs(b.lo[k]), std::fabs(b.hi[k])));
  const double delta = 1e-5 * scale;
  std::vector<std::array<double, 4>> box(objs.size());
  std::vector<std::vector<std::array<double, 2>>> hull(objs.size());
  double umin = INFINITY, umax = -INFINITY, vmin = INFINITY, vmax = -INFINITY;
  for (size_t i = 0; i < objs.size(); ++i) {
    const ObjBox& b = objs[i];
    if (b.always) {
      out->off_grid |= 1ull << i;
      continue;
    }
    hull[i] = convex_hull_2d([&] {
      std::vector<std::array<double, 2>> q(8);
      for (int c = 0; c < 8; ++c) q[(size_t)c] = {dot3(b.corner[c], e1), dot3(b.corner[c], e2)};
      return q;
    }());
    double bu0 = INFINITY, bu1 = -INFINITY, bv0 = INFINITY, bv1 = -INFINITY;
    for (int c = 0; c < 8; ++c) {
      const double p[3] = {(c & 1) ? b.hi[0] : b.lo[0], (c & 2) ? b.hi[1] : b.lo[1], (c & 4) ? b.hi[2] : b.lo[2]};
      const double pu = dot3(p, e1), pv = dot3(p, e2);
      bu0 = std::min(bu0, pu);
      bu1 = std::max(bu1, pu);
      bv0 = std::min(bv0, pv);
      bv1 = std::max(bv1, pv);
    }
    box[i] = {bu0 - delta, bu1 + delta, bv0 - delta, bv1 + delta};
    umin = std::min(umin, box[i][0]);
    umax = std::max(umax, box[i][1]);
    vmin = std::min(vmin, box[i][2]);
    vmax = std::max(vmax, box[i][3]);
  }
  LightGrid& g = out->g;
  for (int k = 0; k < 3; ++k) {
    g.e1[k] = (float)e1[k];
    g.e2[k] = (float)e2[k];
  }
  g.rmax = (float)(50.0 * scale);
  if (!(umin <= umax)) {  // only unbounded objects: a 1x1 grid of the always-set
    g.u0 = g.v0 = 0.0f;
    g.inv_h = 1.0f;
    g.gu = g.gv = 1;
    out->masks.assign(1, out->off_grid);
    return true;
  }
  const double du = std::max(umax - umin, 1e-30), dv = std::max(vmax - vmin, 1e-30);
  const double h = std::max(du, dv) / 256.0;  // 256 cells along the longer side
  const int gu = std::max(1, std::min(256, (int)std::ceil(du / h)));
  const int gv = std::max(1, std::min(256, (int)std::ceil(dv / h)));
  g.u0 = (float)umin;
  g.v0 = (float)vmin;
  g.inv_h = (float)(1.0 / h);
  g.gu = gu;
  g.gv = gv;
  const double ih = (double)g.inv_h;
  out->masks.assign((size_t)gu * (size_t)gv, out->off_grid);
  for (size_t i = 0; i < objs.size(); ++i) {
    if (objs[i].always) continue;
    const int c0 = std::max(0, (int)std::floor((box[i][0] - (double)g.u0) * ih));
    const int c1 = std::min(gu - 1, (int)std::floor((box[i][1] - (double)g.u0) * ih));
    const int r0 = std::max(0, (int)std::floor((box[i][2] - (double)g.v0) * ih));
    const int r1 = std::min(gv - 1, (int)std::floor((box[i][3] - (double)g.v0) * ih));
    // cells meeting the projected hull of the object box's world corners
    // (grown by delta): a shadow ray can only reach the object through its
    // projection, which the hull of the box's projection contains
    const double hc = 1.0 / ih;
    for (int rr = r0; rr <= r1; ++rr)
      for (int cc = c0; cc <= c1; ++cc) {
        const double cu0 = (double)g.u0 + cc * hc - delta, cv0 = (double)g.v0 + rr * hc - delta;
        if (hull[i].size() < 3 || hull_meets_box(hull[i], cu0, cv0, cu0 + hc + 2 * delta, cv0 + hc + 2 * delta))
          out->masks[(size_t)rr * (size_t)gu + (size_t)cc] |= 1ull << i;
      }
  }
  return true;
}

}  // namespace rtmi

// Test entry points (tests/test_bins_cpu.py; not part of include/rtmi.h): the
// builders on a plain face array, face i's record offset = 64 * i.
namespace {
std::vector<rtmi::BinTri> test_tris(const double* v9, int64_t nf) {
  std::vector<rtmi::BinTri> t((size_t)std::max<int64_t>(0, nf));
  for (int64_t i = 0; i < nf; ++i) {
    for (int a = 0; a < 3; ++a)
      for (int k = 0; k < 3; ++k) t[(size_t)i].v[a][k] = v9[9 * i + 3 * a + k];
    t[(size_t)i].rec = (int32_t)(64 * i);
  }
  return t;
}
}  // namespace

extern "C" int64_t rtmi_test_pixel_bins(const double* v9, int64_t nf, const double o2w[16], const double w2o[16],
                                        const double c2w[16], double fov, int32_t w, int32_t h, int32_t* off,
                                        int32_t* ent, int64_t ent_cap) {
  rtmi::PixelBinsHost hb;
  const char* why = "";
  if (!rtmi::build_pixel_bins(test_tris(v9, nf), o2w, w2o, c2w, fov, w, h, &hb, &why)) return -1;
  if ((int64_t)hb.ent.size() > ent_cap) return -2;
  std::copy(hb.off.begin(), hb.off.end(), off);
  std::copy(hb.ent.begin(), hb.ent.end(), ent);
  return (int64_t)hb.off.back();
}

// hdr: e1[3], u0, e2[3], v0, inv_h, rmax, gu, gv (as floats)
extern "C" int64_t rtmi_test_light_grid(const double* v9, int64_t nf, const double w2o[16], const double dir[3],
                                        float* hdr, int32_t* off, int64_t off_cap, int32_t* ent, int64_t ent_cap) {
  rtmi::LightGridHost lg;
  const char* why = "";
  if (!rtmi::build_light_grid(test_tris(v9, nf), w2o, dir, &lg, &why)) return -1;
  if ((int64_t)lg.off.size() > off_cap || (int64_t)lg.ent.size() > ent_cap) return -2;
  const rtmi::LightGrid& g = lg.g;
  const float h[12] = {g.e1[0], g.e1[1], g.e1[2], g.u0, g.e2[0], g.e2[1], g.e2[2], g.v0,
                       g.inv_h, g.rmax, (float)g.gu, (float)g.gv};
  std::copy(h, h + 12, hdr);
  std::copy(lg.off.begin(), lg.off.end(), off);
  std::copy(lg.ent.begin(), lg.ent.end(), ent);
  return (int64_t)lg.off.back();
}

// Per-pixel shadow lists of a one-mesh + planes scene (the arguments of
// rtmi_test_shadow_skips): sl_out = w * h * nl * 2 (start, count; -1: none),
// ent_out (cap entries) = face record offsets (64 x leaf-order index; the
// test's faces in input order). Returns the number of lists, -1 on failure,
// -2 if ent_cap is too small.
extern "C" int64_t rtmi_test_shadow_lists(const double* v9, int64_t nf, const double o2w[16], const double w2o[16],
                                          const double c2w[16], double fov, int32_t w, int32_t h, const double* planes,
                                          int32_t nplanes, const double* dirs, int32_t nl, double bias, int32_t* sl_out,
                                          int32_t* ent_out, int64_t ent_cap) {
  const std::vector<rtmi::BinTri> tris = test_tris(v9, nf);
  rtmi::PixelBinsHost hb;
  const char* why = "";
  if (!rtmi::build_pixel_bins(tris, o2w, w2o, c2w, fov, w, h, &hb, &why)) return -1;
  std::vector<rtmi::GridOcc> occ((size_t)nl);
  std::vector<rtmi::LightGridHost> hosts((size_t)nl);
  for (int l = 0; l < nl; ++l) {
    if (rtmi::build_light_grid(tris, w2o, dirs + 3 * l, &hosts[(size_t)l], &why)) {
      rtmi::grid_occupancy(hosts[(size_t)l], &occ[(size_t)l]);
      occ[(size_t)l].lists = &hosts[(size_t)l];
    }
  }
  std::vector<rtmi::SkipPlane> pl((size_t)nplanes);
  for (int k = 0; k < nplanes; ++k) {
    std::copy(planes + 32 * k, planes + 32 * k + 16, pl[(size_t)k].o2w);
    std::copy(planes + 32 * k + 16, planes + 32 * k + 32, pl[(size_t)k].w2o);
  }
  std::vector<uint32_t> sk;
  std::vector<int32_t> sl, ent;
  if (!rtmi::build_shadow_skips(hb.off, pl, w2o, occ, c2w, fov, w, h, bias, &sk, &why, &sl, &ent, nl)) return -1;
  if ((int64_t)ent.size() > ent_cap) return -2;
  std::copy(sl.begin(), sl.end(), sl_out);
  std::copy(ent.begin(), ent.end(), ent_out);
  int64_t n = 0;
  for (size_t i = 1; i < sl.size(); i += 2) n += sl[i] >= 0;
  return n;
}

// Shadow skips of a one-mesh + planes scene: planes[k] = o2w[16], w2o[16];
// dirs: nl distant-light directions. out: (w * h + 3) / 4 dwords. Returns the
// number of pixels with any skip bit, or -1.
extern "C" int64_t rtmi_test_shadow_skips(const double* v9, int64_t nf, const double o2w[16], const double w2o[16],
                                          const double c2w[16], double fov, int32_t w, int32_t h, const double* planes,
                                          int32_t nplanes, const double* dirs, int32_t nl, double bias, uint32_t* out) {
  const std::vector<rtmi::BinTri> tris = test_tris(v9, nf);
  rtmi::PixelBinsHost hb;
  const char* why = "";
  if (!rtmi::build_pixel_bins(tris, o2w, w2o, c2w, fov, w, h, &hb, &why)) return -1;
  std::vector<rtmi::GridOcc> occ((size_t)nl);
  for (int l = 0; l < nl; ++l) {
    rtmi::LightGridHost lg;
    if (rtmi::build_light_grid(tris, w2o, dirs + 3 * l, &lg, &why)) rtmi::grid_occupancy(lg, &occ[(size_t)l]);
  }
  std::vector<rtmi::SkipPlane> pl((size_t)nplanes);
  for (int k = 0; k < nplanes; ++k) {
    std::copy(planes + 32 * k, planes + 32 * k + 16, pl[(size_t)k].o2w);
    std::copy(planes + 32 * k + 16, planes + 32 * k + 32, pl[(size_t)k].w2o);
  }
  std::vector<uint32_t> sk;
  if (!rtmi::build_shadow_skips(hb.off, pl, w2o, occ, c2w, fov, w, h, bias, &sk, &why)) return -1;
  std::copy(sk.begin(), sk.end(), out);
  int64_t n = 0;
  for (int64_t i = 0; i < (int64_t)w * h; ++i) n += (sk[(size_t)(i >> 2)] >> (8 * (i & 3)) & 0xffu) != 0u;
  return n;
}
