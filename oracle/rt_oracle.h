/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (parity checker + bench.py cpu_baseline).
 * Never linked, loaded or called by the product library (librtmi.so).
 *
 * fp64 CPU restatement of johnnovak/nim-raytracer's per-pixel trace/shade
 * path. See rt_oracle.c for the per-function reference citations and the
 * pinning status (DESIGN.md "Oracle").
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include "../include/rtmi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_scene oracle_scene;

oracle_scene *oracle_scene_create(const rt_scene_desc *desc);
void oracle_scene_destroy(oracle_scene *s);
/* Switch mesh intersection from the reference's brute-force face loop to a
 * per-ray fp64 BVH with the same answers (the "CPU same-BVH" baseline). */
int oracle_scene_build_bvh(oracle_scene *s);

/* renderLine (renderer.nim:162-211) for one row. fb is w*h*3 float32. */
int oracle_render_line(const oracle_scene *s, const rt_options *o, float *fb,
                       int32_t y, int32_t step, int32_t max_step,
                       rt_stats *out);

/* The CLI driver's scanline pool (raytracer.nim:67-109 over
 * workerpool.nim:161-226): `nthreads` workers pull row indices from a shared
 * queue and call renderLine; Stats are summed. rows == NULL means all rows
 * 0..height-1. Returns wall seconds through *seconds (may be NULL). */
int oracle_render_rows_mt(const oracle_scene *s, const rt_options *o,
                          float *fb, const int32_t *rows, int32_t nrows,
                          int32_t step, int32_t max_step, int32_t nthreads,
                          rt_stats *out, double *seconds);

/* ---- known-answer-test entry points ----------------------------------- */
/* solveQuadratic (mathutils.nim:25-29) incl. the `/2*a` precedence. */
void oracle_solve_quadratic(double a, double b, double c, double *t1,
                            double *t2);
/* castPrimaryRay (renderer.nim:31-44): orig[4], dir[4], invdir[3]. */
void oracle_cast_primary_ray(int32_t w, int32_t h, double x, double y,
                             double fov, const double c2w[16], double orig[4],
                             double dir[4]);
/* rayTriangleIntersectFast (geom.nim:283-336); v* are xyz. */
double oracle_ray_triangle(const double orig[4], const double dir[4],
                           const double v0[3], const double v1[3],
                           const double v2[3]);
/* AABB.intersect (geom.nim:76-96). */
double oracle_aabb_intersect(const double vmin[3], const double vmax[3],
                             const double orig[4], const double dir[4]);
/* Sphere.intersect (geom.nim:215-237). */
double oracle_sphere_intersect(double r, const double orig[4],
                               const double dir[4]);
/* trace (renderer.nim:47-67) of a world-space ray; returns object index or
 * -1, *t_hit, *tri_hit (mesh face index or -1). */
int32_t oracle_trace(const oracle_scene *s, const double orig[4],
                     const double dir[4], double t_near, double *t_hit,
                     int64_t *tri_hit, rt_stats *stats);
/* The (m, m) sample table of a stochastic antialias kind for pixel (x, y):
 * sx/sy hold m*m offsets in the reference's p[j*m + i] order. */
void oracle_sample_table(int32_t kind, int32_t m, uint64_t seed, int32_t x,
                         int32_t y, double *sx, double *sy);
/* calcPixelNoSampling / calcPixel (renderer.nim:132-159), fp64 colour. */
void oracle_calc_pixel(const oracle_scene *s, const rt_options *o, int32_t x,
                       int32_t y, double rgb[3], rt_stats *stats);
/* linearToSRGB (color.nim:17-22) + writePpm's outvalue (framebuf.nim:64-68)
 * for one component: clamp, optional sRGB, round(c * maxval). */
int32_t oracle_ppm_outvalue(float v, int32_t bits, int32_t srgb);
/* ImageRGBA.copyFrom's per-component value (src/utils/image.nim:45-54). */
uint8_t oracle_rgba_component(float v);

#ifdef __cplusplus
}
#endif

#endif
