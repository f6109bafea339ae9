/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * fp64 CPU restatement of johnnovak/nim-raytracer's per-pixel trace/shade hot
 * path (the parity checker for tests/ and the timed CPU baseline of bench.py's
 * cpu_baseline leg). The product library librtmi.so never links, loads or
 * calls anything in oracle/.
 *
 * Pinning. The reference is Nim and depends on an un-vendored `nim-glm-fork`
 * (nim.cfg:1); there is no Nim toolchain in this image, so the reference
 * cannot be built or run. This restatement is pinned by
 * the known-answer vectors the reference's own sources hold
 * (tests/test_oracle_kats.py):
 *   - quadratic KAT, src/utils/mathutils.nim:34-45 (rel 1e-15);
 *   - castPrimaryRay / glm post-multiply KAT, test/boxtest.nim:31-41 with
 *     src/data/scenes/boxtest.nim:28-37;
 *   - Moller-Trumbore triangle, test/geomtest2.nim:9-15, test/meshperftest.nim:9-15;
 *   - AABB ray, test/geomtest.cpp:83-87; framebuffer round trip,
 *     src/utils/framebuf.nim:106-119; bunny fixture test/bunny.geom.
 * glm arithmetic beyond those vectors (Y-axis rotation, inverse, summation
 * order of Mat4*Vec4 and dot) follows the standard GLM definitions and is
 * "parity unpinned" beyond the KATs. The reference builds with -ffast-math
 * (src/nim.cfg:2); this oracle deliberately does not (IEEE order, no FMA
 * contraction: compiled with -ffp-contract=off), so it defines one exact
 * answer the device fp64 path must reproduce.
 *
 * Nim semantics kept literally: min(x,y) = (x <= y ? x : y) and
 * max(x,y) = (y <= x ? x : y) (Nim system.nim float min/max), float->int is
 * truncation, `a / 2*a` is `(a/2)*a`.
 */
#include "rt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define NEG_INF (-INFINITY)
#define POS_INF (INFINITY)
#define PI_D 3.14159265358979323846

typedef struct { double x, y, z, w; } v4;
typedef struct { double x, y, z; } v3;

static inline double nmin(double x, double y) { return x <= y ? x : y; }
static inline double nmax(double x, double y) { return y <= x ? x : y; }

/* glm vec4 helpers. Mat4 * Vec4 = sum_i column_i * v[i], accumulated from a
 * zero vector in column order (generic glm matrix-vector product). */
static inline v4 mat_mul_v4(const double m[16], v4 v) {
  v4 r = {0.0, 0.0, 0.0, 0.0};
  const double vv[4] = {v.x, v.y, v.z, v.w};
  for (int c = 0; c < 4; ++c) {
    r.x = r.x + m[c * 4 + 0] * vv[c];
    r.y = r.y + m[c * 4 + 1] * vv[c];
    r.z = r.z + m[c * 4 + 2] * vv[c];
    r.w = r.w + m[c * 4 + 3] * vv[c];
  }
  return r;
}
static inline v4 v4_add(v4 a, v4 b) { v4 r = {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; return r; }
static inline v4 v4_sub(v4 a, v4 b) { v4 r = {a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; return r; }
static inline v4 v4_scale(v4 a, double s) { v4 r = {a.x * s, a.y * s, a.z * s, a.w * s}; return r; }
static inline double v4_dot(v4 a, v4 b) {
  double r = 0.0;
  r = r + a.x * b.x; r = r + a.y * b.y; r = r + a.z * b.z; r = r + a.w * b.w;
  return r;
}
static inline v4 v4_normalize(v4 a) {
  const double len = sqrt(v4_dot(a, a));
  v4 r = {a.x / len, a.y / len, a.z / len, a.w / len};
  return r;
}
static inline v3 v3_cross(v3 a, v3 b) {
  v3 r = {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
  return r;
}
static inline v3 v3_normalize(v3 a) {
  double d = 0.0;
  d = d + a.x * a.x; d = d + a.y * a.y; d = d + a.z * a.z;
  const double len = sqrt(d);
  v3 r = {a.x / len, a.y / len, a.z / len};
  return r;
}

/* mathutils.sign (src/utils/mathutils.nim:12-18). */
static inline double nsign(double x) { return x > 0 ? 1.0 : (x < 0 ? -1.0 : 0.0); }

/* Ray / initRay (src/renderer/geom.nim:32-48). */
typedef struct {
  v4 orig, dir;
  int depth;
  double inv[3];
  int sign[3];
  int64_t tri_hit; /* Ray.triangleHit: face index or -1 (nil) */
} ray_t;

static inline ray_t init_ray(v4 orig, v4 dir, int depth) {
  ray_t r;
  r.orig = orig;
  r.dir = dir;
  r.depth = depth;
  r.inv[0] = 1.0 / dir.x;
  r.inv[1] = 1.0 / dir.y;
  r.inv[2] = 1.0 / dir.z;
  r.sign[0] = r.inv[0] < 0;
  r.sign[1] = r.inv[1] < 0;
  r.sign[2] = r.inv[2] < 0;
  r.tri_hit = -1;
  return r;
}

/* AABB.intersect (geom.nim:76-96): Ize robust slab test. Returns tmin (may
 * be negative: the caller treats that as a miss) or -inf. */
static double aabb_intersect(const v4 b[2], const ray_t *r) {
  double tmin = NEG_INF, tmax = POS_INF;
  const double txmin = (b[r->sign[0]].x - r->orig.x) * r->inv[0];
  const double txmax = (b[1 - r->sign[0]].x - r->orig.x) * r->inv[0];
  const double tymin = (b[r->sign[1]].y - r->orig.y) * r->inv[1];
  const double tymax = (b[1 - r->sign[1]].y - r->orig.y) * r->inv[1];
  const double tzmin = (b[r->sign[2]].z - r->orig.z) * r->inv[2];
  const double tzmax = (b[1 - r->sign[2]].z - r->orig.z) * r->inv[2];
  tmin = nmax(tzmin, nmax(tymin, nmax(txmin, tmin)));
  tmax = nmin(tzmax, nmin(tymax, nmin(txmax, tmax)));
  tmax *= 1.0000000000000004;
  return tmin <= tmax ? tmin : NEG_INF;
}

/* Sphere.intersect (geom.nim:215-237), incl. the `/ 2*a` precedence. */
static double sphere_intersect(double radius, const ray_t *r) {
  const double a = r->dir.x * r->dir.x + r->dir.y * r->dir.y + r->dir.z * r->dir.z;
  const double b = 2 * (r->dir.x * r->orig.x + r->dir.y * r->orig.y + r->dir.z * r->orig.z);
  const double c = r->orig.x * r->orig.x + r->orig.y * r->orig.y + r->orig.z * r->orig.z -
                   radius * radius;
  const double delta = b * b - 4 * a * c;
  if (delta >= 0.0) {
    const double t1 = (-b - nsign(b) * sqrt(delta)) / 2 * a;
    const double t2 = c / (a * t1);
    return nmin(t1, t2);
  }
  return NEG_INF;
}

/* Plane.intersect (geom.nim:240-248): plane y = 0, normal (0,1,0). */
static double plane_intersect(const ray_t *r) {
  const v4 n = {0.0, 1.0, 0.0, 0.0};
  const double denom = v4_dot(n, r->dir);
  if (fabs(denom) > 1e-6) return -v4_dot(r->orig, n) / denom;
  return NEG_INF;
}

/* rayTriangleIntersectFast (geom.nim:283-336): single-sided Moller-Trumbore,
 * absolute det cull 1e-6, no t > 0 test (done by the caller). */
static double ray_triangle(v4 o, v4 d, const double *v0, const double *v1,
                           const double *v2) {
  const double v0v1x = v1[0] - v0[0], v0v1y = v1[1] - v0[1], v0v1z = v1[2] - v0[2];
  const double v0v2x = v2[0] - v0[0], v0v2y = v2[1] - v0[1], v0v2z = v2[2] - v0[2];
  const double pvecx = d.y * v0v2z - d.z * v0v2y;
  const double pvecy = d.z * v0v2x - d.x * v0v2z;
  const double pvecz = d.x * v0v2y - d.y * v0v2x;
  const double det = v0v1x * pvecx + v0v1y * pvecy + v0v1z * pvecz;
  if (det < 0.000001) return NEG_INF;
  const double inv_det = 1 / det;
  const double tvecx = o.x - v0[0], tvecy = o.y - v0[1], tvecz = o.z - v0[2];
  const double u = (tvecx * pvecx + tvecy * pvecy + tvecz * pvecz) * inv_det;
  if (u < 0 || u > 1) return NEG_INF;
  const double qvecx = tvecy * v0v1z - tvecz * v0v1y;
  const double qvecy = tvecz * v0v1x - tvecx * v0v1z;
  const double qvecz = tvecx * v0v1y - tvecy * v0v1x;
  const double v = (d.x * qvecx + d.y * qvecy + d.z * qvecz) * inv_det;
  if (v < 0 || u + v > 1) return NEG_INF;
  return (v0v2x * qvecx + v0v2y * qvecy + v0v2z * qvecz) * inv_det;
}

/* ---- scene --------------------------------------------------------------- */

/* Same-BVH CPU baseline (SURVEY.md 8(d) "CPU same-BVH"): a per-ray fp64
 * BVH over the mesh, built by oracle_scene_build_bvh. count > 0: leaf over
 * order[first, first + count); else children left / right. */
typedef struct {
  double lo[3], hi[3];
  int32_t left, right, first, count;
} obvh_node;

typedef struct {
  int64_t nv, nf;
  double *vertices; /* nv*3 */
  int32_t *faces;   /* nf*3 */
  double *normals;  /* nf*3 face normals */
  v4 aabb[2];       /* calcAABB (geom.nim:175-188) */
  obvh_node *bvh;   /* NULL: brute force (the reference's loop) */
  int32_t *order;
  int32_t nbvh;
} oracle_mesh;

struct oracle_scene {
  int32_t nobj, nlight, nmesh;
  rt_object_desc *objects;
  rt_light_desc *lights;
  oracle_mesh *meshes;
  double fov;
  double c2w[16];
  double bg[3];
};

oracle_scene *oracle_scene_create(const rt_scene_desc *d) {
  if (!d || d->num_objects < 0 || d->num_lights < 0 || d->num_meshes < 0) return NULL;
  oracle_scene *s = (oracle_scene *)calloc(1, sizeof(oracle_scene));
  s->nobj = d->num_objects;
  s->nlight = d->num_lights;
  s->nmesh = d->num_meshes;
  s->objects = (rt_object_desc *)calloc((size_t)s->nobj + 1, sizeof(rt_object_desc));
  s->lights = (rt_light_desc *)calloc((size_t)s->nlight + 1, sizeof(rt_light_desc));
  s->meshes = (oracle_mesh *)calloc((size_t)s->nmesh + 1, sizeof(oracle_mesh));
  if (s->nobj) memcpy(s->objects, d->objects, sizeof(rt_object_desc) * (size_t)s->nobj);
  if (s->nlight) memcpy(s->lights, d->lights, sizeof(rt_light_desc) * (size_t)s->nlight);
  s->fov = d->fov;
  memcpy(s->c2w, d->camera_to_world, sizeof(s->c2w));
  memcpy(s->bg, d->bg_color, sizeof(s->bg));
  for (int32_t i = 0; i < s->nobj; ++i) {
    if (s->objects[i].type == RT_MESH &&
        (s->objects[i].mesh < 0 || s->objects[i].mesh >= s->nmesh)) {
      oracle_scene_destroy(s);
      return NULL;
    }
  }
  for (int32_t m = 0; m < s->nmesh; ++m) {
    const rt_mesh_desc *md = &d->meshes[m];
    oracle_mesh *om = &s->meshes[m];
    om->nv = md->num_vertices;
    om->nf = md->num_faces;
    om->vertices = (double *)malloc(sizeof(double) * 3 * (size_t)(om->nv + 1));
    om->faces = (int32_t *)malloc(sizeof(int32_t) * 3 * (size_t)(om->nf + 1));
    om->normals = (double *)malloc(sizeof(double) * 3 * (size_t)(om->nf + 1));
    memcpy(om->vertices, md->vertices, sizeof(double) * 3 * (size_t)om->nv);
    memcpy(om->faces, md->faces, sizeof(int32_t) * 3 * (size_t)om->nf);
    for (int64_t f = 0; f < om->nf * 3; ++f) {
      if (om->faces[f] < 0 || om->faces[f] >= om->nv) {
        oracle_scene_destroy(s);
        return NULL;
      }
    }
    if (md->normals) {
      memcpy(om->normals, md->normals, sizeof(double) * 3 * (size_t)om->nf);
    } else {
      /* calcNormals (src/loaders/obj.nim:65-84). */
      for (int64_t f = 0; f < om->nf; ++f) {
        const double *p0 = &om->vertices[3 * om->faces[3 * f + 0]];
        const double *p1 = &om->vertices[3 * om->faces[3 * f + 1]];
        const double *p2 = &om->vertices[3 * om->faces[3 * f + 2]];
        v3 a = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
        v3 b = {p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2]};
        v3 n = v3_normalize(v3_cross(a, b));
        om->normals[3 * f + 0] = n.x;
        om->normals[3 * f + 1] = n.y;
        om->normals[3 * f + 2] = n.z;
      }
    }
    /* calcAABB (geom.nim:175-188) over every vertex. */
    v4 vmin = {POS_INF, POS_INF, POS_INF, 1.0}, vmax = {NEG_INF, NEG_INF, NEG_INF, 1.0};
    for (int64_t v = 0; v < om->nv; ++v) {
      const double *p = &om->vertices[3 * v];
      if (p[0] < vmin.x) vmin.x = p[0];
      if (p[1] < vmin.y) vmin.y = p[1];
      if (p[2] < vmin.z) vmin.z = p[2];
      if (p[0] > vmax.x) vmax.x = p[0];
      if (p[1] > vmax.y) vmax.y = p[1];
      if (p[2] > vmax.z) vmax.z = p[2];
    }
    om->aabb[0] = vmin;
    om->aabb[1] = vmax;
  }
  return s;
}

void oracle_scene_destroy(oracle_scene *s) {
  if (!s) return;
  for (int32_t m = 0; m < s->nmesh; ++m) {
    free(s->meshes[m].vertices);
    free(s->meshes[m].faces);
    free(s->meshes[m].normals);
    free(s->meshes[m].bvh);
    free(s->meshes[m].order);
  }
  free(s->meshes);
  free(s->objects);
  free(s->lights);
  free(s);
}

/* TriangleMesh.intersect (geom.nim:339-358): mesh AABB gate (a ray starting
 * inside the box "misses"), then brute force over faces in index order,
 * strict `<` so the lowest face index wins ties. */
static double mesh_intersect(const oracle_mesh *m, ray_t *r) {
  if (aabb_intersect(m->aabb, r) < 0) return NEG_INF;
  double tmin = POS_INF;
  for (int64_t f = 0; f < m->nf; ++f) {
    const int32_t *fi = &m->faces[3 * f];
    const double t = ray_triangle(r->orig, r->dir, &m->vertices[3 * fi[0]],
                                  &m->vertices[3 * fi[1]], &m->vertices[3 * fi[2]]);
    if (t >= 0 && t < tmin) {
      tmin = t;
      r->tri_hit = f;
    }
  }
  return tmin;
}

/* ---- same-BVH baseline ------------------------------------------------- */
/* Binned SAH (16 bins, <= 4 faces per leaf, median fallback) over fp64 face
 * bounds inflated by 2^-30 of the mesh scale, so a face the exact
 * Moller-Trumbore test hits is never culled by a box. The traversal keeps
 * the brute-force loop's answer exactly: a face replaces the best when
 * t >= 0 and (t < best or t == best with a lower face index), and a box is
 * skipped only when its entry distance exceeds the best (ties visited).
 * tests/test_oracle_bvh.py checks image + Stats equality with brute force. */
typedef struct {
  const oracle_mesh *m;
  double *blo, *bhi, *cen; /* per-face bounds / centroids */
  int32_t *idx;
  obvh_node *nodes;
  int32_t nnodes, cap;
  double eps;
} obvh_builder;

static int32_t obvh_new(obvh_builder *B) {
  if (B->nnodes == B->cap) {
    B->cap = B->cap ? 2 * B->cap : 1024;
    B->nodes = (obvh_node *)realloc(B->nodes, sizeof(obvh_node) * (size_t)B->cap);
  }
  return B->nnodes++;
}

static int32_t obvh_build(obvh_builder *B, int32_t b, int32_t e) {
  const int32_t me = obvh_new(B);
  double lo[3] = {POS_INF, POS_INF, POS_INF}, hi[3] = {NEG_INF, NEG_INF, NEG_INF};
  double clo[3] = {POS_INF, POS_INF, POS_INF}, chi[3] = {NEG_INF, NEG_INF, NEG_INF};
  for (int32_t i = b; i < e; ++i) {
    const int32_t f = B->idx[i];
    for (int a = 0; a < 3; ++a) {
      lo[a] = fmin(lo[a], B->blo[3 * f + a]);
      hi[a] = fmax(hi[a], B->bhi[3 * f + a]);
      clo[a] = fmin(clo[a], B->cen[3 * f + a]);
      chi[a] = fmax(chi[a], B->cen[3 * f + a]);
    }
  }
  for (int a = 0; a < 3; ++a) {
    B->nodes[me].lo[a] = lo[a] - B->eps;
    B->nodes[me].hi[a] = hi[a] + B->eps;
  }
  const int32_t n = e - b;
  if (n <= 4) {
    B->nodes[me].first = b;
    B->nodes[me].count = n;
    B->nodes[me].left = B->nodes[me].right = -1;
    return me;
  }
  int axis = 0;
  for (int a = 1; a < 3; ++a)
    if (chi[a] - clo[a] > chi[axis] - clo[axis]) axis = a;
  int32_t mid = -1;
  if (chi[axis] > clo[axis]) { /* binned SAH on the widest centroid axis */
    enum { NB = 16 };
    int32_t cnt[NB] = {0};
    double blo[NB][3], bhi[NB][3];
    for (int k = 0; k < NB; ++k)
      for (int a = 0; a < 3; ++a) { blo[k][a] = POS_INF; bhi[k][a] = NEG_INF; }
    const double scale = NB / (chi[axis] - clo[axis]);
    for (int32_t i = b; i < e; ++i) {
      const int32_t f = B->idx[i];
      int k = (int)((B->cen[3 * f + axis] - clo[axis]) * scale);
      k = k < 0 ? 0 : (k >= NB ? NB - 1 : k);
      cnt[k]++;
      for (int a = 0; a < 3; ++a) {
        blo[k][a] = fmin(blo[k][a], B->blo[3 * f + a]);
        bhi[k][a] = fmax(bhi[k][a], B->bhi[3 * f + a]);
      }
    }
    double best = POS_INF;
    int best_k = -1;
    for (int k = 0; k < NB - 1; ++k) { /* split after bin k */
      double l_lo[3] = {POS_INF, POS_INF, POS_INF}, l_hi[3] = {NEG_INF, NEG_INF, NEG_INF};
      double r_lo[3] = {POS_INF, POS_INF, POS_INF}, r_hi[3] = {NEG_INF, NEG_INF, NEG_INF};
      int32_t nl = 0, nr = 0;
      for (int j = 0; j < NB; ++j) {
        double *L = j <= k ? l_lo : r_lo, *H = j <= k ? l_hi : r_hi;
        if (j <= k) nl += cnt[j]; else nr += cnt[j];
        for (int a = 0; a < 3; ++a) { L[a] = fmin(L[a], blo[j][a]); H[a] = fmax(H[a], bhi[j][a]); }
      }
      if (!nl || !nr) continue;
      const double al = (l_hi[0] - l_lo[0]) * (l_hi[1] - l_lo[1]) + (l_hi[1] - l_lo[1]) * (l_hi[2] - l_lo[2]) +
                        (l_hi[2] - l_lo[2]) * (l_hi[0] - l_lo[0]);
      const double ar = (r_hi[0] - r_lo[0]) * (r_hi[1] - r_lo[1]) + (r_hi[1] - r_lo[1]) * (r_hi[2] - r_lo[2]) +
                        (r_hi[2] - r_lo[2]) * (r_hi[0] - r_lo[0]);
      const double cost = al * nl + ar * nr;
      if (cost < best) { best = cost; best_k = k; }
    }
    if (best_k >= 0) {
      int32_t i = b, j = e - 1;
      while (i <= j) {
        const int32_t f = B->idx[i];
        int k = (int)((B->cen[3 * f + axis] - clo[axis]) * scale);
        k = k < 0 ? 0 : (k >= NB ? NB - 1 : k);
        if (k <= best_k) { ++i; } else { const int32_t t = B->idx[i]; B->idx[i] = B->idx[j]; B->idx[j] = t; --j; }
      }
      mid = i;
    }
  }
  if (mid <= b || mid >= e) mid = b + n / 2; /* degenerate: split the list */
  const int32_t l = obvh_build(B, b, mid);
  const int32_t r = obvh_build(B, mid, e);
  B->nodes[me].left = l;
  B->nodes[me].right = r;
  B->nodes[me].first = 0;
  B->nodes[me].count = 0;
  return me;
}

int oracle_scene_build_bvh(oracle_scene *s) {
  for (int32_t mi = 0; mi < s->nmesh; ++mi) {
    oracle_mesh *m = &s->meshes[mi];
    if (m->bvh || m->nf <= 0) continue;
    obvh_builder B;
    memset(&B, 0, sizeof B);
    B.m = m;
    B.blo = (double *)malloc(sizeof(double) * 3 * (size_t)m->nf);
    B.bhi = (double *)malloc(sizeof(double) * 3 * (size_t)m->nf);
    B.cen = (double *)malloc(sizeof(double) * 3 * (size_t)m->nf);
    B.idx = (int32_t *)malloc(sizeof(int32_t) * (size_t)m->nf);
    double mag = 0.0;
    for (int64_t f = 0; f < m->nf; ++f) {
      B.idx[f] = (int32_t)f;
      for (int a = 0; a < 3; ++a) {
        double lo = POS_INF, hi = NEG_INF;
        for (int k = 0; k < 3; ++k) {
          const double x = m->vertices[3 * m->faces[3 * f + k] + a];
          lo = fmin(lo, x);
          hi = fmax(hi, x);
        }
        B.blo[3 * f + a] = lo;
        B.bhi[3 * f + a] = hi;
        B.cen[3 * f + a] = 0.5 * (lo + hi);
        mag = fmax(mag, fmax(fabs(lo), fabs(hi)));
      }
    }
    B.eps = ldexp(mag, -30) + 1e-300;
    obvh_build(&B, 0, (int32_t)m->nf);
    m->bvh = B.nodes;
    m->nbvh = B.nnodes;
    m->order = B.idx;
    free(B.blo);
    free(B.bhi);
    free(B.cen);
  }
  return 0;
}

/* Entry distance of a conservative slab test (NaN products from 0 * inf are
 * ignored by fmin/fmax, i.e. never cull); +inf on a miss. */
static double obvh_enter(const obvh_node *nd, const ray_t *r) {
  double tn = NEG_INF, tf = POS_INF;
  const double o[3] = {r->orig.x, r->orig.y, r->orig.z};
  for (int a = 0; a < 3; ++a) {
    const double t0 = (nd->lo[a] - o[a]) * r->inv[a], t1 = (nd->hi[a] - o[a]) * r->inv[a];
    tn = fmax(tn, fmin(t0, t1));
    tf = fmin(tf, fmax(t0, t1));
  }
  tf = tf * (1.0 + 1e-12) + 1e-300;
  return (tn <= tf && tf >= 0.0) ? tn : POS_INF;
}

static double mesh_intersect_bvh(const oracle_mesh *m, ray_t *r) {
  if (aabb_intersect(m->aabb, r) < 0) return NEG_INF; /* the reference's gate */
  double tmin = POS_INF;
  int64_t best = -1;
  int32_t stack[128];
  int sp = 0;
  stack[sp++] = 0;
  if (obvh_enter(&m->bvh[0], r) == POS_INF) return tmin;
  while (sp) {
    /* entry distances are re-tested at pop: the best may have shrunk */
    const obvh_node *nd = &m->bvh[stack[--sp]];
    if (obvh_enter(nd, r) > tmin) continue;
    if (nd->count > 0) {
      for (int32_t i = nd->first; i < nd->first + nd->count; ++i) {
        const int32_t f = m->order[i];
        const int32_t *fi = &m->faces[3 * (int64_t)f];
        const double t = ray_triangle(r->orig, r->dir, &m->vertices[3 * fi[0]],
                                      &m->vertices[3 * fi[1]], &m->vertices[3 * fi[2]]);
        if (t >= 0 && (t < tmin || (t == tmin && f < best))) {
          tmin = t;
          best = f;
        }
      }
    } else {
      /* +inf = the box is missed: never pushed (tmin may still be +inf) */
      const double tl = obvh_enter(&m->bvh[nd->left], r), tr = obvh_enter(&m->bvh[nd->right], r);
      const int near_left = tl <= tr;
      const int32_t nn = near_left ? nd->left : nd->right, fn = near_left ? nd->right : nd->left;
      const double tnn = near_left ? tl : tr, tfn = near_left ? tr : tl;
      if (tfn != POS_INF && tfn <= tmin) stack[sp++] = fn; /* far first, near popped next */
      if (tnn != POS_INF && tnn <= tmin) stack[sp++] = nn;
    }
  }
  if (best >= 0) r->tri_hit = best;
  return tmin;
}

static double object_intersect(const oracle_scene *s, const rt_object_desc *ob, ray_t *r) {
  switch (ob->type) {
    case RT_SPHERE: return sphere_intersect(ob->radius, r);
    case RT_PLANE: return plane_intersect(r);
    case RT_BOX: { /* Box.intersect = aabb.intersect (geom.nim:251-252) */
      const v4 b[2] = {{ob->box_min[0], ob->box_min[1], ob->box_min[2], 0.0},
                       {ob->box_max[0], ob->box_max[1], ob->box_max[2], 0.0}};
      return aabb_intersect(b, r);
    }
    case RT_MESH: {
      const oracle_mesh *m = &s->meshes[ob->mesh];
      return m->bvh ? mesh_intersect_bvh(m, r) : mesh_intersect(m, r);
    }
    default: return NEG_INF; /* Geometry.intersect base (geom.nim:213) */
  }
}

/* trace (renderer.nim:47-67): linear closest hit in scene order. */
static int32_t trace(const oracle_scene *s, ray_t *ray, double t_near, double *t_out,
                     rt_stats *st) {
  double tmin = t_near;
  int32_t objmin = -1;
  for (int32_t i = 0; i < s->nobj; ++i) {
    const rt_object_desc *ob = &s->objects[i];
    ray_t ro = init_ray(mat_mul_v4(ob->world_to_object, ray->orig),
                        mat_mul_v4(ob->world_to_object, ray->dir), 1);
    const double t = object_intersect(s, ob, &ro);
    st->num_intersection_tests++;
    if (t >= 0 && t < tmin) {
      tmin = t;
      objmin = i;
      ray->tri_hit = ro.tri_hit;
      st->num_intersection_hits++;
    }
  }
  *t_out = tmin;
  return objmin;
}

/* normal(*) (geom.nim:361-379). */
static v4 object_normal(const rt_object_desc *ob, v4 hit) {
  switch (ob->type) {
    case RT_SPHERE: {
      v4 h = {hit.x, hit.y, hit.z, 0.0};
      return v4_normalize(h);
    }
    case RT_PLANE: {
      v4 n = {0.0, 1.0, 0.0, 0.0};
      return n;
    }
    case RT_BOX: {
      const v4 vmin = {ob->box_min[0], ob->box_min[1], ob->box_min[2], 0.0};
      const v4 vmax = {ob->box_max[0], ob->box_max[1], ob->box_max[2], 0.0};
      const v4 c = v4_scale(v4_add(vmin, vmax), 0.5);
      const v4 p = v4_sub(hit, c);
      const v4 d = v4_scale(v4_sub(vmin, vmax), 0.5);
      const double bias = 1.000001;
      v4 n = {(double)(int64_t)(p.x / fabs(d.x) * bias), (double)(int64_t)(p.y / fabs(d.y) * bias),
              (double)(int64_t)(p.z / fabs(d.z) * bias), 0.0};
      return v4_normalize(n);
    }
    default: {
      v4 z = {0.0, 0.0, 0.0, 0.0};
      return z;
    }
  }
}

/* getShadingInfo (light.nim:43-62). */
typedef struct {
  v4 light_dir;
  double intensity[3];
  double distance;
} shading_info;

static shading_info shading_info_for(const rt_light_desc *l, v4 p) {
  shading_info si;
  if (l->type == RT_POINT_LIGHT) {
    const v4 pos = {l->pos[0], l->pos[1], l->pos[2], 1.0};
    v4 ld = v4_sub(p, pos);
    const double r2 = v4_dot(ld, ld);
    ld = v4_normalize(ld);
    si.light_dir = ld;
    for (int k = 0; k < 3; ++k) si.intensity[k] = l->color[k] * l->intensity / (4 * PI_D * r2);
    si.distance = sqrt(r2);
  } else {
    const v4 dir = {l->dir[0], l->dir[1], l->dir[2], 0.0};
    si.light_dir = dir;
    for (int k = 0; k < 3; ++k) si.intensity[k] = l->color[k] * l->intensity;
    si.distance = POS_INF;
  }
  return si;
}

/* shade (renderer.nim:71-127) with shadeDiffuse (shader.nim:12-17). */
static void shade(const oracle_scene *s, const rt_options *o, ray_t *ray, int32_t obj,
                  double t_hit, double out[3], rt_stats *st) {
  if (obj < 0) {
    out[0] = s->bg[0]; out[1] = s->bg[1]; out[2] = s->bg[2];
    return;
  }
  const rt_object_desc *ob = &s->objects[obj];
  const v4 hit_w = v4_add(ray->orig, v4_scale(ray->dir, t_hit));
  const v4 hit_o = mat_mul_v4(ob->world_to_object, hit_w);
  v4 n;
  if (ray->tri_hit < 0) {
    n = mat_mul_v4(ob->object_to_world, object_normal(ob, hit_o));
  } else {
    const double *fn = &s->meshes[ob->mesh].normals[3 * ray->tri_hit];
    const v4 nrm = {fn[0], fn[1], fn[2], 0.0};
    n = mat_mul_v4(ob->object_to_world, nrm);
  }
  double res[3] = {0.0, 0.0, 0.0};
  for (int32_t li = 0; li < s->nlight; ++li) {
    const shading_info si = shading_info_for(&s->lights[li], hit_w);
    const v4 light_dir = v4_scale(si.light_dir, -1);
    ray_t sr = init_ray(v4_add(hit_w, v4_scale(n, o->bias)), light_dir, 1);
    st->num_shadow_rays++;
    double ts;
    const int32_t shadow_hit = trace(s, &sr, si.distance, &ts, st);
    if (shadow_hit < 0) {
      const double ndl = nmax(0.0, v4_dot(n, v4_scale(si.light_dir, -1)));
      for (int k = 0; k < 3; ++k) res[k] = res[k] + ob->albedo[k] / PI_D * si.intensity[k] * ndl;
    }
  }
  const double refl = ob->reflection;
  if (refl > 0.0 && ray->depth <= o->max_ray_depth) {
    const v4 i = ray->dir;
    const v4 r = v4_sub(i, v4_scale(n, 2 * v4_dot(n, i)));
    ray_t rr = init_ray(v4_add(hit_w, v4_scale(r, o->bias)), r, ray->depth + 1);
    st->num_reflection_rays++;
    double tr;
    const int32_t objr = trace(s, &rr, POS_INF, &tr, st);
    double rc[3];
    if (objr >= 0) {
      shade(s, o, &rr, objr, tr, rc, st);
    } else {
      rc[0] = s->bg[0]; rc[1] = s->bg[1]; rc[2] = s->bg[2];
    }
    for (int k = 0; k < 3; ++k) res[k] = (1.0 - refl) * res[k] + refl * rc[k];
  }
  out[0] = res[0]; out[1] = res[1]; out[2] = res[2];
}

/* castPrimaryRay (renderer.nim:31-44); degToRad = d * (PI/180) (Nim math). */
static ray_t cast_primary_ray(int32_t w, int32_t h, double x, double y, double fov,
                              const double c2w[16]) {
  const double r = (double)w / (double)h;
  const double f = tan(fov * (PI_D / 180.0) / 2);
  const double cx = ((2 * x * r) / (double)w - r) * f;
  const double cy = (1 - 2 * y / (double)h) * f;
  const v4 origin = {0.0, 0.0, 0.0, 1.0};
  const v4 d = {cx, cy, -1.0, 0.0};
  return init_ray(mat_mul_v4(c2w, origin), mat_mul_v4(c2w, v4_normalize(d)), 1);
}

static void sample(const oracle_scene *s, const rt_options *o, double px, double py,
                   double out[3], rt_stats *st) {
  ray_t ray = cast_primary_ray(o->width, o->height, px, py, s->fov, s->c2w);
  st->num_primary_rays++;
  double t;
  const int32_t obj = trace(s, &ray, POS_INF, &t, st);
  shade(s, o, &ray, obj, t, out, st);
}

/* ---- stochastic samplers (sampling.nim:21-113) -------------------------- */
/* The reference draws from Nim's `random`, seeded from the clock
 * (renderer.nim:215 `randomize()`), so its jittered images are not
 * reproducible. Here every draw is a pure function of (options.seed, pixel,
 * draw index) — a SplitMix64 counter RNG — so the device kernels (which
 * build a pixel's table in parallel) reproduce it exactly; the ORDER of the
 * draws is the reference's loop order:
 *   jitteredGrid   sampling.nim:21-33  2 draws per (j, i), row-major;
 *   multiJittered  sampling.nim:39-76  2 per (j, i) canonical, then one per
 *                                      (j, i) for the x shuffle, then one per
 *                                      (i, j) (i outer) for the y shuffle;
 *   correlatedMJ   sampling.nim:79-113 same canonical, one per row j (x), one
 *                                      per column i (y).
 * random(x) = u * x with u uniform in [0, 1) (53 bits); `.int` truncates. */
static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
static uint64_t pixel_key(uint64_t seed, int32_t x, int32_t y) {
  return mix64(seed ^ mix64(((uint64_t)(uint32_t)y << 32) | (uint32_t)x));
}
static double draw_u(uint64_t key, uint64_t k) {
  return (double)(mix64(key + (k + 1) * 0x9E3779B97F4A7C15ULL) >> 11) * (1.0 / 9007199254740992.0);
}

/* p[j*m + i] of jitteredGrid / multiJittered / correlatedMultiJittered (m, m). */
static void sample_table(int32_t kind, int32_t m, uint64_t key, double *sx, double *sy) {
  const int32_t n = m;
  const double xs = 1.0 / (double)n, ys = 1.0 / (double)m;
  if (kind == RT_AA_JITTERED) {
    for (int32_t j = 0; j < m; ++j)
      for (int32_t i = 0; i < n; ++i) {
        const int32_t e = j * m + i;
        sx[e] = (double)i * xs + draw_u(key, 2 * (uint64_t)e) * xs;
        sy[e] = (double)j * ys + draw_u(key, 2 * (uint64_t)e + 1) * ys;
      }
    return;
  }
  for (int32_t j = 0; j < n; ++j)
    for (int32_t i = 0; i < m; ++i) {
      const int32_t e = j * m + i;
      sx[e] = ((double)i + ((double)j + draw_u(key, 2 * (uint64_t)e)) * xs) * ys;
      sy[e] = ((double)j + ((double)i + draw_u(key, 2 * (uint64_t)e + 1)) * ys) * xs;
    }
  const uint64_t bx = 2 * (uint64_t)m * n;
  if (kind == RT_AA_MULTI_JITTERED) {
    const uint64_t by = bx + (uint64_t)m * n;
    for (int32_t j = 0; j < n; ++j)
      for (int32_t i = 0; i < m; ++i) {
        const int32_t k = j + (int32_t)(draw_u(key, bx + (uint64_t)j * m + i) * (double)(n - j));
        const double t = sx[j * m + i];
        sx[j * m + i] = sx[k * m + i];
        sx[k * m + i] = t;
      }
    for (int32_t i = 0; i < m; ++i)
      for (int32_t j = 0; j < n; ++j) {
        const int32_t k = i + (int32_t)(draw_u(key, by + (uint64_t)i * n + j) * (double)(m - i));
        const double t = sy[j * m + i];
        sy[j * m + i] = sy[j * m + k];
        sy[j * m + k] = t;
      }
  } else { /* correlated: one k per row (x) and per column (y) */
    const uint64_t by = bx + (uint64_t)n;
    for (int32_t j = 0; j < n; ++j) {
      const int32_t k = j + (int32_t)(draw_u(key, bx + (uint64_t)j) * (double)(n - j));
      for (int32_t i = 0; i < m; ++i) {
        const double t = sx[j * m + i];
        sx[j * m + i] = sx[k * m + i];
        sx[k * m + i] = t;
      }
    }
    for (int32_t i = 0; i < m; ++i) {
      const int32_t k = i + (int32_t)(draw_u(key, by + (uint64_t)i) * (double)(m - i));
      for (int32_t j = 0; j < n; ++j) {
        const double t = sy[j * m + i];
        sy[j * m + i] = sy[j * m + k];
        sy[j * m + k] = t;
      }
    }
  }
}

void oracle_sample_table(int32_t kind, int32_t m, uint64_t seed, int32_t x, int32_t y, double *sx, double *sy) {
  sample_table(kind, m, pixel_key(seed, x, y), sx, sy);
}

/* calcPixelNoSampling / calcPixel (renderer.nim:132-159) with grid()
 * (sampling.nim:5-18, incl. yoffs = xs*0.5) or the stochastic tables. */
void oracle_calc_pixel(const oracle_scene *s, const rt_options *o, int32_t x, int32_t y,
                       double rgb[3], rt_stats *st) {
  if (o->aa_kind == RT_AA_NONE) {
    sample(s, o, (double)x, (double)y, rgb, st);
    return;
  }
  const int32_t m = o->grid_size, n = o->grid_size;
  const double xs = 1.0 / (double)n, ys = 1.0 / (double)m;
  const double xoffs = xs * 0.5, yoffs = xs * 0.5;
  double acc[3] = {0.0, 0.0, 0.0};
  const int32_t len = m * n;
  double *tx = NULL, *ty = NULL;
  if (o->aa_kind != RT_AA_GRID) {
    tx = (double *)malloc(sizeof(double) * 2 * (size_t)len);
    ty = tx + len;
    sample_table(o->aa_kind, m, pixel_key(o->seed, x, y), tx, ty);
  }
  for (int32_t k = 0; k < len; ++k) {
    const int32_t j = k / m, i = k % m; /* p[j*m + i] */
    const double sx = tx ? tx[k] : (double)i * xs + xoffs, sy = ty ? ty[k] : (double)j * ys + yoffs;
    double c[3];
    sample(s, o, (double)x + sx, (double)y + sy, c, st);
    for (int q = 0; q < 3; ++q) acc[q] = acc[q] + c[q];
  }
  free(tx);
  const double inv = 1.0 / (double)len;
  for (int q = 0; q < 3; ++q) rgb[q] = acc[q] * inv;
}

static int is_pow2(int32_t v) { return v > 0 && (v & (v - 1)) == 0; }

int oracle_render_line(const oracle_scene *s, const rt_options *o, float *fb, int32_t y,
                       int32_t step, int32_t max_step, rt_stats *out) {
  if (!s || !o || !fb) return RT_E_INVALID;
  if (!is_pow2(step) || !is_pow2(max_step) || max_step < step) return RT_E_INVALID;
  if (y < 0 || y >= o->height) return RT_E_INVALID;
  if (o->aa_kind < RT_AA_NONE || o->aa_kind > RT_AA_CORRELATED_MULTI_JITTERED) return RT_E_INVALID;
  if (o->aa_kind != RT_AA_NONE && (o->grid_size < 1 || o->grid_size > 256)) return RT_E_INVALID;
  rt_stats st;
  memset(&st, 0, sizeof(st));
  const int32_t w = o->width, h = o->height;
  for (int32_t x = 0; x < w; x += step) {
    if (step < max_step) {
      const int32_t mask = step * 2 - 1;
      if ((x & mask) == 0 && (y & mask) == 0) continue;
    }
    double c[3];
    oracle_calc_pixel(s, o, x, y, c, &st);
    const float cf[3] = {(float)c[0], (float)c[1], (float)c[2]};
    if (step > 1) {
      for (int32_t i = x; i < (x + step < w ? x + step : w); ++i)
        for (int32_t j = y; j < (y + step < h ? y + step : h); ++j) {
          float *p = &fb[((size_t)j * w + i) * 3];
          p[0] = cf[0]; p[1] = cf[1]; p[2] = cf[2];
        }
    } else {
      float *p = &fb[((size_t)y * w + x) * 3];
      p[0] = cf[0]; p[1] = cf[1]; p[2] = cf[2];
    }
  }
  if (out) {
    out->num_primary_rays += st.num_primary_rays;
    out->num_intersection_tests += st.num_intersection_tests;
    out->num_intersection_hits += st.num_intersection_hits;
    out->num_shadow_rays += st.num_shadow_rays;
    out->num_reflection_rays += st.num_reflection_rays;
  }
  return RT_OK;
}

/* ---- scanline pool (raytracer.nim:67-109, workerpool.nim:161-226) ------- */
typedef struct {
  const oracle_scene *s;
  const rt_options *o;
  float *fb;
  const int32_t *rows;
  int32_t nrows, step, max_step;
  pthread_mutex_t lock;
  int32_t next;
  rt_stats total;
  int err;
} pool_t;

static void *pool_worker(void *arg) {
  pool_t *p = (pool_t *)arg;
  rt_stats local;
  memset(&local, 0, sizeof(local));
  int err = RT_OK;
  for (;;) {
    pthread_mutex_lock(&p->lock);
    const int32_t k = p->next++;
    pthread_mutex_unlock(&p->lock);
    if (k >= p->nrows) break;
    const int32_t y = p->rows ? p->rows[k] : k;
    const int e = oracle_render_line(p->s, p->o, p->fb, y, p->step, p->max_step, &local);
    if (e != RT_OK) err = e;
  }
  pthread_mutex_lock(&p->lock);
  p->total.num_primary_rays += local.num_primary_rays;
  p->total.num_intersection_tests += local.num_intersection_tests;
  p->total.num_intersection_hits += local.num_intersection_hits;
  p->total.num_shadow_rays += local.num_shadow_rays;
  p->total.num_reflection_rays += local.num_reflection_rays;
  if (err != RT_OK) p->err = err;
  pthread_mutex_unlock(&p->lock);
  return NULL;
}

int oracle_render_rows_mt(const oracle_scene *s, const rt_options *o, float *fb,
                          const int32_t *rows, int32_t nrows, int32_t step, int32_t max_step,
                          int32_t nthreads, rt_stats *out, double *seconds) {
  if (!s || !o || !fb) return RT_E_INVALID;
  if (!rows) nrows = o->height;
  if (nthreads < 1) nthreads = 1;
  pool_t p;
  memset(&p, 0, sizeof(p));
  p.s = s; p.o = o; p.fb = fb; p.rows = rows; p.nrows = nrows;
  p.step = step; p.max_step = max_step;
  pthread_mutex_init(&p.lock, NULL);
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int32_t i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, pool_worker, &p);
  for (int32_t i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  free(th);
  pthread_mutex_destroy(&p.lock);
  if (seconds) *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
  if (out) {
    out->num_primary_rays += p.total.num_primary_rays;
    out->num_intersection_tests += p.total.num_intersection_tests;
    out->num_intersection_hits += p.total.num_intersection_hits;
    out->num_shadow_rays += p.total.num_shadow_rays;
    out->num_reflection_rays += p.total.num_reflection_rays;
  }
  return p.err;
}

/* ---- KAT entry points ------------------------------------------------------ */
void oracle_solve_quadratic(double a, double b, double c, double *t1, double *t2) {
  /* quadraticDelta / solveQuadratic (mathutils.nim:22-29). */
  const double delta = b * b - 4 * a * c;
  const double r1 = (-b - nsign(b) * sqrt(delta)) / 2 * a;
  *t1 = r1;
  *t2 = c / (a * r1);
}

void oracle_cast_primary_ray(int32_t w, int32_t h, double x, double y, double fov,
                             const double c2w[16], double orig[4], double dir[4]) {
  const ray_t r = cast_primary_ray(w, h, x, y, fov, c2w);
  orig[0] = r.orig.x; orig[1] = r.orig.y; orig[2] = r.orig.z; orig[3] = r.orig.w;
  dir[0] = r.dir.x; dir[1] = r.dir.y; dir[2] = r.dir.z; dir[3] = r.dir.w;
}

double oracle_ray_triangle(const double orig[4], const double dir[4], const double v0[3],
                           const double v1[3], const double v2[3]) {
  const v4 o = {orig[0], orig[1], orig[2], orig[3]};
  const v4 d = {dir[0], dir[1], dir[2], dir[3]};
  return ray_triangle(o, d, v0, v1, v2);
}

double oracle_aabb_intersect(const double vmin[3], const double vmax[3], const double orig[4],
                             const double dir[4]) {
  const v4 b[2] = {{vmin[0], vmin[1], vmin[2], 1.0}, {vmax[0], vmax[1], vmax[2], 1.0}};
  const v4 o = {orig[0], orig[1], orig[2], orig[3]};
  const v4 d = {dir[0], dir[1], dir[2], dir[3]};
  const ray_t r = init_ray(o, d, 1);
  return aabb_intersect(b, &r);
}

double oracle_sphere_intersect(double radius, const double orig[4], const double dir[4]) {
  const v4 o = {orig[0], orig[1], orig[2], orig[3]};
  const v4 d = {dir[0], dir[1], dir[2], dir[3]};
  const ray_t r = init_ray(o, d, 1);
  return sphere_intersect(radius, &r);
}

int32_t oracle_trace(const oracle_scene *s, const double orig[4], const double dir[4],
                     double t_near, double *t_hit, int64_t *tri_hit, rt_stats *stats) {
  const v4 o = {orig[0], orig[1], orig[2], orig[3]};
  const v4 d = {dir[0], dir[1], dir[2], dir[3]};
  ray_t r = init_ray(o, d, 1);
  rt_stats local;
  memset(&local, 0, sizeof(local));
  const int32_t obj = trace(s, &r, t_near, t_hit, stats ? stats : &local);
  if (tri_hit) *tri_hit = r.tri_hit;
  return obj;
}

/* linearToSRGB (color.nim:17-22) + writePpm.outvalue (framebuf.nim:74-78). */
uint8_t oracle_rgba_component(float v) {
  /* image.nim:51-53: round(fb.data[i] * 0xff).uint8 — a float32 product
   * (the literal converts to float32), Nim round on float32 (roundf), then
   * the uint8 conversion. No clamp: for results outside [0, 255] the
   * reference either raises (range checks on) or, in a release build on
   * x86-64, keeps the low 8 bits of the int32 conversion (cvttss2si: NaN and
   * |x| >= 2^31 give INT32_MIN). That release behaviour is restated here;
   * no reference test pins it. */
  const float r = roundf(v * 255.0f);
  const int32_t i = (r >= -2147483648.0f && r < 2147483648.0f) ? (int32_t)r : INT32_MIN;
  return (uint8_t)((uint32_t)i & 0xffu);
}

int32_t oracle_ppm_outvalue(float v, int32_t bits, int32_t srgb) {
  /* maxval = float32(2^bits - 1) (framebuf.nim:58); c = clamp(v, 0, 1) is
   * float32; linearToSRGB (color.nim:17-22) evaluates in float64 (its `a` is
   * a float64 let) and returns float32; `round(c * maxval)` is a float32
   * product rounded half away from zero (Nim round on float32). */
  const float maxval = (float)((1 << bits) - 1);
  float c = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
  if (c != c) c = 0.0f; /* NaN: the reference's Natural() conversion raises; 0 here */
  if (srgb) {
    const double a = 0.055, cd = (double)c;
    c = (float)(cd <= 0.0031308 ? 12.92 * cd : (1 + a) * pow(cd, 1 / 2.4) - a);
  }
  return (int32_t)roundf(c * maxval);
}
