// rt_bins_geom.h — float64 geometry shared by the host bin builders
// (rt_bins.cpp, the tests' reference) and the per-frame device builders
// (rt_frame.hip). Both are compiled with -ffp-contract=off, so host and
// device form every bound with the same roundings and build the same lists.
#pragma once
#include <hip/hip_runtime.h>

#include <math.h>

namespace rtmi {
namespace bg {

// glm column-major: m[c*4 + r]
__host__ __device__ inline void xform_point(const double m[16], const double p[3], double out[3]) {
  for (int r = 0; r < 3; ++r) out[r] = m[0 * 4 + r] * p[0] + m[1 * 4 + r] * p[1] + m[2 * 4 + r] * p[2] + m[3 * 4 + r];
}
__host__ __device__ inline void xform_dir(const double m[16], const double d[3], double out[3]) {
  for (int r = 0; r < 3; ++r) out[r] = m[0 * 4 + r] * d[0] + m[1 * 4 + r] * d[1] + m[2 * 4 + r] * d[2];
}
__host__ __device__ inline double dot3(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
__host__ __device__ inline void cross3(const double a[3], const double b[3], double o[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
__host__ __device__ inline double norm3(const double a[3]) { return sqrt(dot3(a, a)); }
__host__ __device__ inline double dmin(double a, double b) { return b < a ? b : a; }
__host__ __device__ inline double dmax(double a, double b) { return a < b ? b : a; }

// The single-sided test rejects det < 1e-6 (geom.nim:306). det is computed
// in float32 from the object-space direction rd and nn = -(e1 x e2); a face
// is left out of a family's bins only when det stays below 1e-6 even with a
// float32 error of 1e-6 * |rd| * |nn| (generous: the test's own rounding is
// ~1e-7 of that).
__host__ __device__ inline bool never_passes(double det_upper, double rd_max, double nlen) {
  return det_upper + 1e-6 * rd_max * nlen < 1e-6;
}

// Separating-axis test of a 2D triangle q[0..5] (x, y pairs) against the box
// [x0, x1] x [y0, y1] (the box axes are the caller's bounding-rectangle
// loop): false only when one triangle edge has all four box corners strictly
// outside it.
__host__ __device__ inline bool tri_meets_box(const double* q, double x0, double y0, double x1, double y1) {
  const double area = (q[2] - q[0]) * (q[5] - q[1]) - (q[3] - q[1]) * (q[4] - q[0]);
  if (!(area != 0.0)) return true;  // degenerate (or NaN): keep
  const double sg = area > 0.0 ? 1.0 : -1.0;
  const double cx[4] = {x0, x1, x0, x1}, cy[4] = {y0, y0, y1, y1};
  for (int k = 0; k < 3; ++k) {
    const int k1 = k == 2 ? 0 : k + 1;
    const double ax = q[2 * k], ay = q[2 * k + 1];
    const double bx = q[2 * k1], by = q[2 * k1 + 1];
    double best = -INFINITY;
    for (int c = 0; c < 4; ++c) best = dmax(best, sg * ((bx - ax) * (cy[c] - ay) - (by - ay) * (cx[c] - ax)));
    if (best < 0.0) return false;
  }
  return true;
}

// Camera-ray bins of one face (build_pixel_bins): the face's projected
// vertices in pixel coordinates (q[6]) and its pixel rectangle (rect[4]:
// x0, x1, y0, y1; x0 = -1: the face gets no bin). Returns false when a vertex
// lies at or behind the camera plane (no bins for this camera).
struct PixCam {
  double o2w[16], w2c[16];  // mesh object -> world, world -> camera
  double co[3];             // camera origin in mesh object space
  double rd_min, rd_max;    // |rd| bounds of a unit world direction in object space
  double cam_a, cam_c;      // the float32 kernel's camera constants (rtmi.cpp fill_fast)
  double margin;            // rt_bins.h kPixelMargin
  int width, height;
};
// The single-sided cull of a face for every camera ray (geom.nim:306): true
// when no camera ray reaching the face's plane can pass det >= 1e-6.
__host__ __device__ inline bool face_is_back(const PixCam& c, const double v[3][3]) {
  double e1[3], e2[3], cr[3], nn[3], dc[3];
  for (int k = 0; k < 3; ++k) {
    e1[k] = v[1][k] - v[0][k];
    e2[k] = v[2][k] - v[0][k];
    dc[k] = v[0][k] - c.co[k];
  }
  cross3(e1, e2, cr);
  for (int k = 0; k < 3; ++k) nn[k] = -cr[k];
  const double nlen = norm3(nn);
  // every camera ray reaching the face's plane has det = |rd| (v0 - C).nn / |P - C|
  const double s = dot3(dc, nn);
  double maxd = 0.0;
  for (int a = 0; a < 3; ++a) {
    const double dv[3] = {v[a][0] - c.co[0], v[a][1] - c.co[1], v[a][2] - c.co[2]};
    maxd = dmax(maxd, norm3(dv));
  }
  return s <= 0.0 && maxd > 0.0 && never_passes(c.rd_min * s / maxd, c.rd_max, nlen);
}
// The face's projected vertices and grown pixel rectangle (rect[0] = -1:
// off screen); false when a vertex lies at or behind the camera plane.
__host__ __device__ inline bool face_project_rect(const PixCam& c, const double v[3][3], double q[6], int rect[4]) {
  rect[0] = rect[1] = rect[2] = rect[3] = -1;
  double xmin = INFINITY, xmax = -INFINITY, ymin = INFINITY, ymax = -INFINITY;
  for (int a = 0; a < 3; ++a) {
    double pw[3], pc[3];
    xform_point(c.o2w, v[a], pw);
    xform_point(c.w2c, pw, pc);
    if (!(pc[2] < -1e-9 * (1.0 + fabs(pc[0]) + fabs(pc[1])))) return false;
    const double px = 0.5 * c.width + (pc[0] / -pc[2]) / c.cam_a;
    const double py = 0.5 * c.height - (pc[1] / -pc[2]) / c.cam_c;
    q[2 * a] = px;
    q[2 * a + 1] = py;
    xmin = dmin(xmin, px);
    xmax = dmax(xmax, px);
    ymin = dmin(ymin, py);
    ymax = dmax(ymax, py);
  }
  const double m = c.margin;
  if (!(xmax + m >= 0.0 && ymax + m >= 0.0 && xmin - m < c.width && ymin - m < c.height)) return true;
  rect[0] = (int)dmax(0.0, floor(xmin - m));
  rect[1] = (int)dmin((double)c.width - 1, floor(xmax + m));
  rect[2] = (int)dmax(0.0, floor(ymin - m));
  rect[3] = (int)dmin((double)c.height - 1, floor(ymax + m));
  return true;
}
__host__ __device__ inline bool face_pixel_rect(const PixCam& c, const double v[3][3], double q[6], int rect[4]) {
  if (face_is_back(c, v)) {  // a back face: in no pixel's list
    rect[0] = rect[1] = rect[2] = rect[3] = -1;
    return true;
  }
  return face_project_rect(c, v, q, rect);
}

// Shadow skips (build_shadow_skips) of one pixel whose camera-ray list is
// empty: bit l set when every shadow ray to distant light l leaving a camera
// hit of the pixel provably meets no face. Per plane (a plane object of the
// scene, y = 0 in its object space), the per-camera constants:
struct SkipPlaneC {
  double oy;        // camera origin's object-space y
  double row[3];    // object-space y of a world direction: row . d
  double n[3];      // world normal (object_to_world * (0, 1, 0), as the kernel's N)
  double tol;       // float32 error allowance of row . d
};
// One light's grid as the skip test reads it: the float32 LightGrid values
// widened, and its occupancy prefix counts ((gu + 1) x (gv + 1)).
struct SkipGrid {
  double e1[3], e2[3], u0, v0, inv_h;
  int gu, gv;
  const int* sat;
};
struct SkipCam {
  double c2w[16], cw[3], mesh_w2o[16];
  double cam_a, cam_c, margin, bias;
  int width, height;
};
// The skip bits (a subset of `have`) shared by every pixel of the rectangle
// [x0, x1] x [y0, y1] — its grown corner rays bound every pixel's — or 0
// when a horizon crosses it. One pixel: x0 = x1, y0 = y1.
__host__ __device__ inline unsigned rect_skip_bits(const SkipCam& c, const SkipPlaneC* planes, int nplanes,
                                                   const SkipGrid* grids, int nl, unsigned have, int x0, int y0,
                                                   int x1, int y1) {
  double dw[4][3];
  for (int k = 0; k < 4; ++k) {
    const double px = (k & 1) ? x1 + 1 + c.margin : x0 - c.margin, py = (k & 2) ? y1 + 1 + c.margin : y0 - c.margin;
    const double dc[3] = {(px - 0.5 * c.width) * c.cam_a, (0.5 * c.height - py) * c.cam_c, -1.0};
    xform_dir(c.c2w, dc, dw[k]);
    const double il = 1.0 / norm3(dw[k]);
    for (int a = 0; a < 3; ++a) dw[k][a] *= il;
  }
  unsigned bits = have;
  for (int k = 0; k < nplanes && bits; ++k) {
    const SkipPlaneC& P = planes[k];
    int hit = 0, miss = 0;
    double t[4] = {0.0, 0.0, 0.0, 0.0};
    for (int q = 0; q < 4; ++q) {
      const double dy = dot3(P.row, dw[q]);
      // the kernel counts a plane hit at t = -oy / dy >= 0 with |dy| > 1e-6
      const double s = P.oy > 0.0 ? -dy : dy;  // > 0: towards the plane
      if (s > P.tol + 1e-6) {
        ++hit;
        t[q] = -P.oy / dy;
      } else if (s < -P.tol) {
        ++miss;
      }
    }
    if (miss == 4) continue;  // no ray of the pixel reaches this plane
    if (hit != 4) return 0u;  // a horizon inside the pixel: unbounded footprint
    for (int l = 0; l < nl; ++l) {
      if (!(bits >> l & 1u)) continue;
      const SkipGrid& g = grids[l];
      double umin = INFINITY, umax = -INFINITY, vmin = INFINITY, vmax = -INFINITY, qmax = 0.0;
      for (int q = 0; q < 4; ++q) {
        // shadow-ray origin: hit + N * bias (renderer.nim:94-101), in mesh space
        const double so[3] = {c.cw[0] + dw[q][0] * t[q] + P.n[0] * c.bias, c.cw[1] + dw[q][1] * t[q] + P.n[1] * c.bias,
                              c.cw[2] + dw[q][2] * t[q] + P.n[2] * c.bias};
        double o[3];
        xform_point(c.mesh_w2o, so, o);
        qmax = dmax(qmax, dmax(fabs(o[0]), dmax(fabs(o[1]), fabs(o[2]))));
        const double u = dot3(o, g.e1), v = dot3(o, g.e2);
        umin = dmin(umin, u);
        umax = dmax(umax, u);
        vmin = dmin(vmin, v);
        vmax = dmax(vmax, v);
      }
      // float32 hit points, transforms, shadow rays and triangle tests: far
      // inside 1e-4 of the magnitudes. A face a shadow ray of the footprint
      // can meet overlaps the grown footprint, so it is listed in a cell
      // the footprint's cell range holds (cells list every face whose grown
      // projection meets them): no cell beyond that range is needed.
#ifndef RTMI_SKIP_CELL_PAD
#define RTMI_SKIP_CELL_PAD 0.0
#endif
      const double mw = 1e-4 * (1.0 + qmax) + 1e-4 * fabs(c.bias);
      const double ih = g.inv_h;
      const double fu0 = (umin - mw - g.u0) * ih - RTMI_SKIP_CELL_PAD, fu1 = (umax + mw - g.u0) * ih + RTMI_SKIP_CELL_PAD;
      const double fv0 = (vmin - mw - g.v0) * ih - RTMI_SKIP_CELL_PAD, fv1 = (vmax + mw - g.v0) * ih + RTMI_SKIP_CELL_PAD;
      if (!(fu1 >= 0.0 && fv1 >= 0.0 && fu0 < g.gu && fv0 < g.gv)) continue;  // off the grid
      if (!isfinite(fu0 + fu1 + fv0 + fv1)) {
        bits &= ~(1u << l);
        continue;
      }
      const int u0 = (int)dmax(0.0, floor(fu0)), u1 = (int)dmin((double)g.gu - 1, floor(fu1));
      const int v0 = (int)dmax(0.0, floor(fv0)), v1 = (int)dmin((double)g.gv - 1, floor(fv1));
      const long long W1 = (long long)g.gu + 1;
      const int n = g.sat[(long long)(v1 + 1) * W1 + u1 + 1] - g.sat[(long long)v0 * W1 + u1 + 1] -
                    g.sat[(long long)(v1 + 1) * W1 + u0] + g.sat[(long long)v0 * W1 + u0];
      if (n != 0) bits &= ~(1u << l);
    }
  }
  return bits;
}
__host__ __device__ inline unsigned pixel_skip_bits(const SkipCam& c, const SkipPlaneC* planes, int nplanes,
                                                    const SkipGrid* grids, int nl, unsigned have, int x, int y) {
  return rect_skip_bits(c, planes, nplanes, grids, nl, have, x, y, x, y);
}

}  // namespace bg
}  // namespace rtmi
