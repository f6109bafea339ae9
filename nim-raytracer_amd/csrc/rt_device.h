// rt_device.h — gfx950 (CDNA4) trace/shade kernels, templated on the
// arithmetic type R (float = performance mode, double = parity mode).
//
// Design (DESIGN.md "Kernels"):
//  * One wave = one tile of pixels x samples. With >= 64 samples per pixel
//    (the benchmark configs) a wave is ONE pixel and its 64 lanes trace 64
//    sub-pixel samples at a time, so the wave's rays are almost perfectly
//    coherent.
//  * Wave-coherent BVH traversal: the node index and the traversal stack are
//    wave-uniform. Node (64 B, both child boxes) and triangle records are
//    fetched with SCALAR loads (s_load through the constant address space),
//    each lane tests the child boxes against its own ray, and __ballot decides
//    which children the wave visits. The stack lives in one VGPR across the
//    64 lanes (entry i in lane i: push = v_cndmask, pop = v_readlane), so
//    there is no per-lane stack, no LDS traffic and no scratch.
//  * Statistics are wave-uniform popcounts of ballots kept in SGPRs and
//    written once per wave (no atomics in the hot loop).
//  * R = double reproduces the oracle's (i.e. the reference's) float64
//    operation order: compiled with -ffp-contract=off, literal glm vec4
//    arithmetic including the w components, IEEE division and sqrt.
#pragma once
#include <hip/hip_runtime.h>

#include "rt_common.h"
#include "rt_sampling.h"

#ifndef RT_CONST
#if defined(__HIP_DEVICE_COMPILE__)
#define RT_CONST __attribute__((address_space(4)))  // scalar (constant) loads
#else
#define RT_CONST
#endif
#endif

namespace rtmi {

template <class T>
__device__ __forceinline__ const RT_CONST T* cptr(const T* p) {
  return (const RT_CONST T*)(p);
}

// Kernel parameters read through a laundered pointer into the kernarg
// segment (as rt_fast.h params()): each field is re-read with a scalar load
// near its use instead of being pinned in SGPRs for the whole kernel (the
// pinned float64 camera matrix and bases spilled ~150 SGPRs into VGPR lanes).
template <class R>
__device__ __forceinline__ const RT_CONST RenderParams<R>& rparams() {
  const RT_CONST RenderParams<R>* q = (const RT_CONST RenderParams<R>*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(q));
  return *q;
}

template <class R> struct Prec;
template <> struct Prec<float> {
  static constexpr bool exact = false;
  __device__ static __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }
  __device__ static __forceinline__ float div(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
  __device__ static __forceinline__ float sqrt(float x) { return __builtin_sqrtf(x); }
  static constexpr float aabb_tmax_scale = 1.00000024f;  // geom.nim:90 (float form)
  static constexpr float node_tmax_scale = 1.0000004f;   // conservative BVH culling
};
template <> struct Prec<double> {
  static constexpr bool exact = true;
  __device__ static __forceinline__ double rcp(double x) { return 1.0 / x; }
  __device__ static __forceinline__ double div(double a, double b) { return a / b; }
  __device__ static __forceinline__ double sqrt(double x) { return __builtin_sqrt(x); }
  static constexpr double aabb_tmax_scale = 1.0000000000000004;  // geom.nim:91
  static constexpr double node_tmax_scale = 1.000000000001;
};

template <class R> struct V3 { R x, y, z; };

// Nim system.nim float min/max (NaN semantics kept).
template <class R> __device__ __forceinline__ R nmin(R x, R y) { return x <= y ? x : y; }
template <class R> __device__ __forceinline__ R nmax(R x, R y) { return y <= x ? x : y; }
// mathutils.sign (mathutils.nim:12-18)
template <class R> __device__ __forceinline__ R nsign(R x) { return x > R(0) ? R(1) : (x < R(0) ? R(-1) : R(0)); }

template <class R> __device__ __forceinline__ R pinf() { return __builtin_huge_val(); }
template <> __device__ __forceinline__ float pinf<float>() { return __builtin_huge_valf(); }

// glm Mat4 * Vec4 (sum of columns scaled by v, accumulated from zero in
// column order). w is 1 for points and 0 for directions; in exact mode the
// w column is multiplied literally, as the reference does.
template <class R, class M>
__device__ __forceinline__ V3<R> xform(const M& m, V3<R> v, R w) {
  V3<R> r;
  if constexpr (Prec<R>::exact) {
    r.x = R(0); r.y = R(0); r.z = R(0);
    r.x = r.x + m[0] * v.x;  r.y = r.y + m[1] * v.x;  r.z = r.z + m[2] * v.x;
    r.x = r.x + m[4] * v.y;  r.y = r.y + m[5] * v.y;  r.z = r.z + m[6] * v.y;
    r.x = r.x + m[8] * v.z;  r.y = r.y + m[9] * v.z;  r.z = r.z + m[10] * v.z;
    r.x = r.x + m[12] * w;   r.y = r.y + m[13] * w;   r.z = r.z + m[14] * w;
  } else {
    r.x = m[0] * v.x + m[4] * v.y + m[8] * v.z + m[12] * w;
    r.y = m[1] * v.x + m[5] * v.y + m[9] * v.z + m[13] * w;
    r.z = m[2] * v.x + m[6] * v.y + m[10] * v.z + m[14] * w;
  }
  return r;
}

// glm Mat4 * Vec4 for an object's matrix of host class xf (DevObject.xf;
// XF_IDENTITY / XF_TRANSLATE: both object matrices have an identity 3x3
// block). In exact mode the literal sum of such a matrix collapses bit for
// bit: row x is (((0 + 1*v.x) + 0*v.y) + 0*v.z) + m[12]*w, and with v.y, v.z
// finite the signed-zero products leave the partial sum 0 + v.x unchanged
// (it is never -0), so the row is (0 + v.x) + m[12] for a point and 0 + v.x
// for a direction (m[12]*0 is another signed zero). The callers pass only
// values that are finite on every lane whose result is used (ray origins and
// directions, hit points of hits, normals); 2-3 float64 operations per row
// instead of 8.
template <class R, bool POINT, class M>
__device__ __forceinline__ V3<R> xform_xf(int xf, const M& m, V3<R> v) {
  if constexpr (Prec<R>::exact) {
    if (xf != XF_GENERAL) {
      if constexpr (POINT) return V3<R>{(R(0) + v.x) + m[12], (R(0) + v.y) + m[13], (R(0) + v.z) + m[14]};
      return V3<R>{R(0) + v.x, R(0) + v.y, R(0) + v.z};
    }
  }
  return xform<R>(m, v, POINT ? R(1) : R(0));
}

// vec4 dot with explicit w terms (exact mode keeps the literal sum order).
template <class R>
__device__ __forceinline__ R dot4(V3<R> a, R aw, V3<R> b, R bw) {
  if constexpr (Prec<R>::exact) {
    R r = R(0);
    r = r + a.x * b.x; r = r + a.y * b.y; r = r + a.z * b.z; r = r + aw * bw;
    return r;
  } else {
    return a.x * b.x + a.y * b.y + a.z * b.z;
  }
}

// normalize of a vec4 direction (w = 0): v / length(v).
template <class R>
__device__ __forceinline__ V3<R> normalize_dir(V3<R> v) {
  const R len = Prec<R>::sqrt(dot4(v, R(0), v, R(0)));
  if constexpr (Prec<R>::exact) {
    return V3<R>{v.x / len, v.y / len, v.z / len};
  } else {
    const R il = R(1) / len;
    return V3<R>{v.x * il, v.y * il, v.z * il};
  }
}

// ---- wave helpers ----------------------------------------------------------
__device__ __forceinline__ unsigned long long ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ unsigned long long popc(unsigned long long m) {
  return (unsigned long long)__popcll(m);
}

// Wave-uniform 32-bit counters (SGPRs), flushed per pixel group into a
// per-lane 64-bit total (lane k holds slot k). Traversal counters (node /
// triangle fetches) are only kept by the instrumented kernel (COUNT).
struct WaveStats {
  unsigned int v[kStatSlots];
};
__device__ __forceinline__ unsigned int popc32(unsigned long long m) { return (unsigned int)__popcll(m); }

// ---- primitive intersections (object space) -------------------------------
// Object-space ray as initRay builds it (geom.nim:41-48).
template <class R>
struct ORay {
  V3<R> o, d, inv;
};

template <class R>
__device__ __forceinline__ ORay<R> init_oray(V3<R> o, V3<R> d) {
  ORay<R> r;
  r.o = o;
  r.d = d;
  r.inv = V3<R>{Prec<R>::rcp(d.x), Prec<R>::rcp(d.y), Prec<R>::rcp(d.z)};
  return r;
}

// AABB.intersect (geom.nim:76-96), returns tmin or -inf.
template <class R>
__device__ __forceinline__ R aabb_ref(V3<R> lo, V3<R> hi, const ORay<R>& r) {
  if constexpr (!Prec<R>::exact) {
    // same test with IEEE min/max instead of the sign-indexed bounds (equal
    // except for NaN slabs, whose Nim semantics only the float64 mode keeps)
    const float ax = (lo.x - r.o.x) * r.inv.x, bx = (hi.x - r.o.x) * r.inv.x;
    const float ay = (lo.y - r.o.y) * r.inv.y, by = (hi.y - r.o.y) * r.inv.y;
    const float az = (lo.z - r.o.z) * r.inv.z, bz = (hi.z - r.o.z) * r.inv.z;
    const float tmin = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    const float tmax = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz)) * Prec<R>::aabb_tmax_scale;
    return tmin <= tmax ? tmin : -pinf<R>();
  }
  const bool sx = r.inv.x < R(0), sy = r.inv.y < R(0), sz = r.inv.z < R(0);
  const R txmin = ((sx ? hi.x : lo.x) - r.o.x) * r.inv.x;
  const R txmax = ((sx ? lo.x : hi.x) - r.o.x) * r.inv.x;
  const R tymin = ((sy ? hi.y : lo.y) - r.o.y) * r.inv.y;
  const R tymax = ((sy ? lo.y : hi.y) - r.o.y) * r.inv.y;
  const R tzmin = ((sz ? hi.z : lo.z) - r.o.z) * r.inv.z;
  const R tzmax = ((sz ? lo.z : hi.z) - r.o.z) * r.inv.z;
  const R tmin = nmax(tzmin, nmax(tymin, nmax(txmin, -pinf<R>())));
  R tmax = nmin(tzmax, nmin(tymax, nmin(txmax, pinf<R>())));
  tmax *= Prec<R>::aabb_tmax_scale;
  return tmin <= tmax ? tmin : -pinf<R>();
}

// Sphere.intersect (geom.nim:215-237), incl. the `/ 2*a` precedence.
template <class R>
__device__ __forceinline__ R sphere_ref(R radius, const ORay<R>& r) {
  const R a = r.d.x * r.d.x + r.d.y * r.d.y + r.d.z * r.d.z;
  const R b = R(2) * (r.d.x * r.o.x + r.d.y * r.o.y + r.d.z * r.o.z);
  const R c = r.o.x * r.o.x + r.o.y * r.o.y + r.o.z * r.o.z - radius * radius;
  const R delta = b * b - R(4) * a * c;
  if (delta >= R(0)) {
    const R t1 = Prec<R>::div(-b - nsign(b) * Prec<R>::sqrt(delta), R(2)) * a;
    const R t2 = Prec<R>::div(c, a * t1);
    return nmin(t1, t2);
  }
  return -pinf<R>();
}

// Plane.intersect (geom.nim:240-248): y = 0, n = (0,1,0,0).
template <class R>
__device__ __forceinline__ R plane_ref(const ORay<R>& r) {
  if constexpr (Prec<R>::exact) {
    // the literal dot4 sums with n = (0, 1, 0, 0) collapse exactly (as in
    // xform_xf: for finite x / z components the signed-zero terms leave
    // 0 + y unchanged): dot(n, d) = 0 + d.y, dot(o, n) = 0 + o.y
    const R denom = R(0) + r.d.y;
    if (fabs(denom) > R(1e-6)) return Prec<R>::div(-(R(0) + r.o.y), denom);
    return -pinf<R>();
  }
  const V3<R> n{R(0), R(1), R(0)};
  const R denom = dot4(n, R(0), r.d, R(0));
  if (fabs(denom) > R(1e-6)) {
    return Prec<R>::div(-dot4(r.o, R(1), n, R(0)), denom);
  }
  return -pinf<R>();
}

// rayTriangleIntersectFast (geom.nim:283-336) over a precomputed record
// (e1 = v1 - v0, e2 = v2 - v0, bitwise what the reference computes). Returns
// the hit t or NaN-free -inf. Single-sided (det < 1e-6 culled).
template <class R, class T>
__device__ __forceinline__ R tri_ref(const T& tri, V3<R> o, V3<R> d) {
  const R v0v1x = tri.e1[0], v0v1y = tri.e1[1], v0v1z = tri.e1[2];
  const R v0v2x = tri.e2[0], v0v2y = tri.e2[1], v0v2z = tri.e2[2];
  const R pvecx = d.y * v0v2z - d.z * v0v2y;
  const R pvecy = d.z * v0v2x - d.x * v0v2z;
  const R pvecz = d.x * v0v2y - d.y * v0v2x;
  const R det = v0v1x * pvecx + v0v1y * pvecy + v0v1z * pvecz;
  const R inv_det = Prec<R>::rcp(det);
  const R tvecx = o.x - R(tri.v0[0]), tvecy = o.y - R(tri.v0[1]), tvecz = o.z - R(tri.v0[2]);
  const R u = (tvecx * pvecx + tvecy * pvecy + tvecz * pvecz) * inv_det;
  const R qvecx = tvecy * v0v1z - tvecz * v0v1y;
  const R qvecy = tvecz * v0v1x - tvecx * v0v1z;
  const R qvecz = tvecx * v0v1y - tvecy * v0v1x;
  const R v = (d.x * qvecx + d.y * qvecy + d.z * qvecz) * inv_det;
  const R t = (v0v2x * qvecx + v0v2y * qvecy + v0v2z * qvecz) * inv_det;
  // det < 1e-6 -> -inf; u < 0 or u > 1 -> -inf; v < 0 or u + v > 1 -> -inf.
  // (The reference's early outs are order-independent predicates; a NaN
  // anywhere makes the final `t >= 0` of the caller false, as in Nim.)
  const bool ok = !(det < R(0.000001)) && !(u < R(0) || u > R(1)) && !(v < R(0) || u + v > R(1));
  return ok ? t : -pinf<R>();
}

// ---- wave-coherent BVH traversal -------------------------------------------
// Closest hit (or any hit) over one mesh for the lanes with `active`, within
// [0, tbest). Must be called from wave-uniform control flow (the stack push
// writes lane `sp`). best_id = original face index of the hit, -1 if none;
// an equal-t hit replaces a larger face index (the reference's brute-force
// loop keeps the lowest index on ties, geom.nim:354).
template <class R>
__device__ __forceinline__ void slab2(const RT_CONST BvhNode& nd, V3<R> o, V3<R> ninv, V3<R> oi,
                                      R tbest, bool active, bool& h0, bool& h1, R& tn0, R& tn1) {
  if constexpr (Prec<R>::exact) {
    const R ax0 = (R(nd.lo0[0]) - o.x) * ninv.x, bx0 = (R(nd.hi0[0]) - o.x) * ninv.x;
    const R ay0 = (R(nd.lo0[1]) - o.y) * ninv.y, by0 = (R(nd.hi0[1]) - o.y) * ninv.y;
    const R az0 = (R(nd.lo0[2]) - o.z) * ninv.z, bz0 = (R(nd.hi0[2]) - o.z) * ninv.z;
    const R ax1 = (R(nd.lo1[0]) - o.x) * ninv.x, bx1 = (R(nd.hi1[0]) - o.x) * ninv.x;
    const R ay1 = (R(nd.lo1[1]) - o.y) * ninv.y, by1 = (R(nd.hi1[1]) - o.y) * ninv.y;
    const R az1 = (R(nd.lo1[2]) - o.z) * ninv.z, bz1 = (R(nd.hi1[2]) - o.z) * ninv.z;
    tn0 = fmax(fmax(fmin(ax0, bx0), fmin(ay0, by0)), fmax(fmin(az0, bz0), R(0)));
    const R tf0 = fmin(fmin(fmax(ax0, bx0), fmax(ay0, by0)), fmin(fmax(az0, bz0), tbest));
    tn1 = fmax(fmax(fmin(ax1, bx1), fmin(ay1, by1)), fmax(fmin(az1, bz1), R(0)));
    const R tf1 = fmin(fmin(fmax(ax1, bx1), fmax(ay1, by1)), fmin(fmax(az1, bz1), tbest));
    h0 = active && tn0 <= tf0 * Prec<R>::node_tmax_scale;
    h1 = active && tn1 <= tf1 * Prec<R>::node_tmax_scale;
  } else {
    const R ax0 = __builtin_fmaf(nd.lo0[0], ninv.x, -oi.x), bx0 = __builtin_fmaf(nd.hi0[0], ninv.x, -oi.x);
    const R ay0 = __builtin_fmaf(nd.lo0[1], ninv.y, -oi.y), by0 = __builtin_fmaf(nd.hi0[1], ninv.y, -oi.y);
    const R az0 = __builtin_fmaf(nd.lo0[2], ninv.z, -oi.z), bz0 = __builtin_fmaf(nd.hi0[2], ninv.z, -oi.z);
    const R ax1 = __builtin_fmaf(nd.lo1[0], ninv.x, -oi.x), bx1 = __builtin_fmaf(nd.hi1[0], ninv.x, -oi.x);
    const R ay1 = __builtin_fmaf(nd.lo1[1], ninv.y, -oi.y), by1 = __builtin_fmaf(nd.hi1[1], ninv.y, -oi.y);
    const R az1 = __builtin_fmaf(nd.lo1[2], ninv.z, -oi.z), bz1 = __builtin_fmaf(nd.hi1[2], ninv.z, -oi.z);
    tn0 = fmaxf(fmaxf(fminf(ax0, bx0), fminf(ay0, by0)), fmaxf(fminf(az0, bz0), 0.0f));
    const R tf0 = fminf(fminf(fmaxf(ax0, bx0), fmaxf(ay0, by0)), fminf(fmaxf(az0, bz0), tbest));
    tn1 = fmaxf(fmaxf(fminf(ax1, bx1), fminf(ay1, by1)), fmaxf(fminf(az1, bz1), 0.0f));
    const R tf1 = fminf(fminf(fmaxf(ax1, bx1), fmaxf(ay1, by1)), fminf(fmaxf(az1, bz1), tbest));
    h0 = active && tn0 <= tf0 * Prec<R>::node_tmax_scale;
    h1 = active && tn1 <= tf1 * Prec<R>::node_tmax_scale;
  }
}

template <class R, bool COUNT>
__device__ __forceinline__ void leaf(const RT_CONST RenderParams<R>& p, int first, int count, bool h,
                                     V3<R> o, V3<R> d, R& tbest, int& best_id, bool& active,
                                     bool early, R stop, WaveStats& ws) {
  using Tri = typename TriOf<R>::type;
  if constexpr (COUNT) {
    ws.v[STAT_TRI_FETCH] += (unsigned int)count;
    ws.v[STAT_LANE_TRIS] += popc32(ballot(h)) * (unsigned int)count;
  }
  for (int k = 0; k < count; ++k) {
    const RT_CONST Tri& tri = cptr(p.tris)[first + k];
    const R t = tri_ref<R>(tri, o, d);
    const int id = tri.id;
    const bool acc = h && t >= R(0) && (t < tbest || (t == tbest && id < best_id));
    if (acc) {
      tbest = t;
      best_id = id;
    }
  }
  // exact shadow early exit (see trace): retire on a found hit at t <= stop
  if (early) active = active && !(best_id >= 0 && tbest <= stop);
}

template <class R, bool COUNT>
__device__ __forceinline__ void traverse(const RT_CONST RenderParams<R>& p, int root, V3<R> o, V3<R> d,
                                         bool active, bool early, R stop, R& tbest, int& best_id,
                                         WaveStats& ws) {
  if (ballot(active) == 0ull || root < 0) return;
  V3<R> ninv, oi;
  if constexpr (Prec<R>::exact) {
    ninv = V3<R>{R(1) / d.x, R(1) / d.y, R(1) / d.z};
    oi = V3<R>{R(0), R(0), R(0)};
  } else {
    // clamp exact-zero components so the fma slab form never sees inf*0
    const float e = 1e-20f;
    const float dx = __builtin_fabsf(d.x) < e ? __builtin_copysignf(e, d.x) : d.x;
    const float dy = __builtin_fabsf(d.y) < e ? __builtin_copysignf(e, d.y) : d.y;
    const float dz = __builtin_fabsf(d.z) < e ? __builtin_copysignf(e, d.z) : d.z;
    ninv = V3<R>{Prec<R>::rcp(dx), Prec<R>::rcp(dy), Prec<R>::rcp(dz)};
    oi = V3<R>{o.x * ninv.x, o.y * ninv.y, o.z * ninv.z};
  }
  const int lane = (int)__lane_id();
  int stack = 0;  // entry i lives in lane i
  int sp = 0;
  int node = root;
  for (int iter = 0; iter < p.max_iters; ++iter) {
    const RT_CONST BvhNode& nd = cptr(p.nodes)[node];
    if constexpr (COUNT) {
      ws.v[STAT_NODE_FETCH] += 1u;
      ws.v[STAT_LANE_NODES] += popc32(ballot(active));
    }
    bool h0, h1;
    R tn0, tn1;
    slab2<R>(nd, o, ninv, oi, tbest, active, h0, h1, tn0, tn1);
    const int c0 = nd.c0, c1 = nd.c1, n0 = nd.n0, n1 = nd.n1;
    // empty children (c < 0, n == 0) are never visited
    unsigned long long m0 = (n0 > 0 || c0 >= 0) ? ballot(h0) : 0ull;
    unsigned long long m1 = (n1 > 0 || c1 >= 0) ? ballot(h1) : 0ull;
    if (n0 > 0 && m0) {
      leaf<R, COUNT>(p, c0, n0, h0, o, d, tbest, best_id, active, early, stop, ws);
      m0 = 0;
    }
    if (n1 > 0 && m1) {
      leaf<R, COUNT>(p, c1, n1, h1, o, d, tbest, best_id, active, early, stop, ws);
      m1 = 0;
    }
    if (early && ballot(active) == 0ull) break;
    if (m0 && m1) {
      const unsigned long long both = m0 & m1;
      const unsigned long long near0 = ballot(h0 && h1 && tn0 <= tn1);
      const bool first0 = popc(near0) * 2 >= popc(both);
      const int near = first0 ? c0 : c1;
      const int far = first0 ? c1 : c0;
      stack = (lane == sp) ? far : stack;
      ++sp;
      node = near;
    } else if (m0) {
      node = c0;
    } else if (m1) {
      node = c1;
    } else {
      if (sp == 0) break;
      --sp;
      node = __builtin_amdgcn_readlane(stack, sp);
    }
  }
}

// ---- binned face lists (k_render_px64: one pixel per wave) ------------------
// The faces at ent[0, n) — a pixel's camera-ray list or a light-grid cell,
// each a TriFast byte offset (rt_frame.h / rt_bins.h) — against the lanes
// with `act`, with the traversal's rules: a face replaces the best hit when
// t >= 0 and (t, face) is below (tbest, best_id), so the result is the
// lexicographic minimum over the listed faces whatever their order — and a
// list holds every face a ray of its family can hit (the builders' float64
// proof, tests/test_bins_cpu.py), so it equals geom.nim:339-358's loop over
// all faces. early: the shadow early exit (a lane retires on a found hit at
// t <= stop, as in leaf()).
template <class R>
__device__ __forceinline__ void list_tris(const RT_CONST RenderParams<R>& p, const int32_t* ent, int n, V3<R> o, V3<R> d,
                                          bool act, bool early, R stop, R& tbest, int& best_id) {
  using Tri = typename TriOf<R>::type;
  for (int k = 0; k < n; ++k) {
    const int off = cptr(ent)[k];
    const RT_CONST Tri& tri = cptr(p.tris)[(off >> 6) - p.tri_rec0];
    const R t = tri_ref<R>(tri, o, d);
    const int id = tri.id;
    const bool acc = act && t >= R(0) && (t < tbest || (t == tbest && id < best_id));
    if (acc) {
      tbest = t;
      best_id = id;
    }
    if (early && (k & 3) == 3) {
      act = act && !(best_id >= 0 && tbest <= stop);
      if (ballot(act) == 0ull) break;
    }
  }
}

// The same search over a cell's float64 shadow records (ShTri64, one
// distant light's fixed direction d): tri_ref's operations with pvec, det and
// invDet read from the record (formed from the same d by k_build_sh64). A
// face whose det fails the cull is skipped (det is the same for every lane),
// and so are qvec / v / t when no lane's u passes (u's test decides the
// reference's second early out; the others are order-independent predicates).
template <class R>
__device__ __forceinline__ void list_sh64(const ShTri64* rec, int n, V3<R> o, V3<R> d, bool act, bool early, R stop,
                                          R& tbest, int& best_id) {
  // LDS staging (the float32 kernels' idea, here for 128-B float64 records):
  // four records = 64 doubles are ONE coalesced vector load (a double per
  // lane) into the wave's LDS slice, read back as broadcasts; the next four
  // are loaded while these are tested (two slices), so the search waits on
  // one load per four faces, not on a scalar load per face.
  __shared__ double stage[4][2][64];  // [wave of a 256-thread block][buffer][double]
  const int lane = (int)__lane_id();
  double* slice = &stage[(threadIdx.x >> 6) & 3][0][0];
  const double* src = (const double*)rec;
  const int nd = n * 16;
  const int ngroups = (n + 3) >> 2;
  double pre = lane < nd ? src[lane] : 0.0;
  for (int g = 0; g < ngroups; ++g) {
    double* buf = slice + (g & 1) * 64;
    buf[lane] = pre;
    // the slice is read by every lane of this wave: LDS operations of one
    // wave complete in order; the barrier keeps the compiler from moving the
    // reads above the write
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (g + 1 < ngroups) {
      const int i = (g + 1) * 64 + lane;
      pre = i < nd ? src[i] : 0.0;
    }
    const int jn = min(4, n - 4 * g);
    for (int j = 0; j < jn; ++j) {
      const double* f = buf + 16 * j;  // ShTri64 layout: v0, e1, e2, pvec, det, inv_det, id
      const R det = f[12];
      if (!(det < R(0.000001))) {
        const R v0v1x = f[3], v0v1y = f[4], v0v1z = f[5];
        const R v0v2x = f[6], v0v2y = f[7], v0v2z = f[8];
        const R inv_det = f[13];
        const R tvecx = o.x - R(f[0]), tvecy = o.y - R(f[1]), tvecz = o.z - R(f[2]);
        const R u = (tvecx * f[9] + tvecy * f[10] + tvecz * f[11]) * inv_det;
        const bool uok = act && !(u < R(0) || u > R(1));
        if (ballot(uok) != 0ull) {
          const R qvecx = tvecy * v0v1z - tvecz * v0v1y;
          const R qvecy = tvecz * v0v1x - tvecx * v0v1z;
          const R qvecz = tvecx * v0v1y - tvecy * v0v1x;
          const R v = (d.x * qvecx + d.y * qvecy + d.z * qvecz) * inv_det;
          const R t = (v0v2x * qvecx + v0v2y * qvecy + v0v2z * qvecz) * inv_det;
          const int id = ((const int32_t*)(f + 14))[0];
          const bool acc = uok && !(v < R(0) || u + v > R(1)) && t >= R(0) && (t < tbest || (t == tbest && id < best_id));
          if (acc) {
            tbest = t;
            best_id = id;
          }
        }
      }
      if (early && j == 3) {  // every fourth face, as list_tris
        act = act && !(best_id >= 0 && tbest <= stop);
        if (ballot(act) == 0ull) return;
      }
    }
  }
}

// The mesh's closest hit for the lanes `in` (past the AABB gate) of a
// one-pixel wave: camera rays (pix >= 0) search the pixel's list unless it
// outgrew its slots, shadow rays to a distant light with a grid search
// their cells (every distinct cell of the wave in turn, each with its own
// lanes); lanes without a list take the BVH.
template <class R, bool COUNT>
__device__ __forceinline__ void mesh_lists(const RT_CONST RenderParams<R>& p, int root, const ORay<R>& r, bool in, bool early,
                                           R stop, int pix, unsigned pinfo, int light, R& tbest, int& best_id,
                                           WaveStats& ws) {
  if (pix >= 0 && p.pix_slots) {
    const unsigned n = pinfo & kPixCount;
    if (n <= (1u << p.slot_lg)) {
      list_tris<R>(p, p.pix_slots + ((size_t)pix << p.slot_lg), (int)n, r.o, r.d, in, early, stop, tbest, best_id);
      return;
    }
  } else if (light >= 0 && p.grids) {
    const RT_CONST LightGrid& G = cptr(p.grids)[light];
    if (G.gu > 0) {
      const R gu = r.o.x * R(G.e1[0]) + r.o.y * R(G.e1[1]) + r.o.z * R(G.e1[2]);
      const R gv = r.o.x * R(G.e2[0]) + r.o.y * R(G.e2[1]) + r.o.z * R(G.e2[2]);
      const R fu = (gu - R(G.u0)) * R(G.inv_h), fv = (gv - R(G.v0)) * R(G.inv_h);
      const bool safe = fmax(fmax(fabs(r.o.x), fabs(r.o.y)), fabs(r.o.z)) <= R(G.rmax);
      const bool on = fu >= R(0) && fu < R(G.gu) && fv >= R(0) && fv < R(G.gv);
      const int bin = safe && on ? G.off_base + (int)fv * G.gu + (int)fu : -1;
      const bool nohit = safe && !on;  // off the grid: no listed face, so no face at all
      unsigned long long todo = ballot(in && bin >= 0);
      while (todo) {
        const int kb = __builtin_amdgcn_readlane(bin, (int)__builtin_ctzll(todo));
        todo &= ~ballot(bin == kb);
        const int b = cptr(p.grid_off)[kb], e = cptr(p.grid_off)[kb + 1];
        if (Prec<R>::exact && p.sh64)
          list_sh64<R>(p.sh64 + G.ent_base + b, e - b, r.o, r.d, in && bin == kb, early, stop, tbest, best_id);
        else
          list_tris<R>(p, p.grid_ent + G.ent_base + b, e - b, r.o, r.d, in && bin == kb, early, stop, tbest, best_id);
      }
      in = in && bin < 0 && !nohit;
    }
  }
  traverse<R, COUNT>(p, root, r.o, r.d, in, early, stop, tbest, best_id, ws);
}

// ---- trace (renderer.nim:47-67) --------------------------------------------
template <class R>
struct Hit {
  int obj;   // -1 = nil
  int tri;   // original face index of a mesh hit, -1 otherwise
  R t;
};

// World -> object space for one object. float32 mode takes the identity /
// translation shortcuts the host classified (DevObject.xf); float64 mode
// always multiplies the full matrix so every rounding matches the oracle.
template <class R>
__device__ __forceinline__ void to_object(const RT_CONST DevObject<R>& ob, V3<R> o, V3<R> d, V3<R>& ro,
                                          V3<R>& rd) {
  if constexpr (!Prec<R>::exact) {
    const int xf = ob.xf;
    if (xf == XF_IDENTITY) {
      ro = o;
      rd = d;
      return;
    }
    if (xf == XF_TRANSLATE) {
      ro = V3<R>{o.x + ob.w2o[12], o.y + ob.w2o[13], o.z + ob.w2o[14]};
      rd = d;
      return;
    }
  }
  ro = xform_xf<R, true>(ob.xf, ob.w2o, o);
  rd = xform_xf<R, false>(ob.xf, ob.w2o, d);
}

// t of an analytic object (plane / sphere / box) in its object space.
template <class R>
__device__ __forceinline__ R analytic_t(const RT_CONST DevObject<R>& ob, int type, ORay<R> r) {
  if (type == GEOM_PLANE) return plane_ref<R>(r);
  if (type == GEOM_SPHERE) return sphere_ref<R>(ob.prm[0], r);
  if (type == GEOM_BOX) {
    r.inv = V3<R>{Prec<R>::rcp(r.d.x), Prec<R>::rcp(r.d.y), Prec<R>::rcp(r.d.z)};
    return aabb_ref<R>(V3<R>{ob.prm[0], ob.prm[1], ob.prm[2]}, V3<R>{ob.prm[4], ob.prm[5], ob.prm[6]}, r);
  }
  return -pinf<R>();
}

// Per-block LDS cache of k_render_px64 (scenes of <= kCacheObj objects and
// <= kCacheLight lights): the values every sample of the frame would compute
// the same way — each object's view of the camera origin, each distant
// light's shadow direction in each object's space (and its reciprocals), each
// plane's world normal — formed once per block with the same operations, so
// the same bits.
constexpr int kCacheObj = 16, kCacheLight = 8;
constexpr int kCacheCamO = 0;                                 // [obj][4]: w2o * (camera origin, 1)
constexpr int kCacheLightD = kCacheCamO + 4 * kCacheObj;      // [light][obj][8]: w2o * (-ldir, 0), 1 / that
constexpr int kCachePlaneN = kCacheLightD + 8 * kCacheObj * kCacheLight;  // [obj][4]: o2w * (0, 1, 0, 0)
// [light][4]: the lean plane's shading term per light (px64_lean_sample):
// albedo/PI * lightIntensity * max(0, N . -lightDir) — sample-invariant for a
// plane under a distant light
constexpr int kCacheLeanTerm = kCachePlaneN + 4 * kCacheObj;
constexpr int kCacheDoubles = kCacheLeanTerm + 4 * kCacheLight;

// Linear closest hit over the scene's objects in order, for lanes with
// `active`; tmin starts at t_near. Wave-uniform control flow only.
//
// Shadow rays (`shadow`) use an EXACT early exit when the scene has one mesh
// object (p.shadow_mesh): the caller needs only whether anything is hit and
// the reference's hit count, in which an object after the mesh counts only
// if its t beats the mesh's closest t. Once a lane holds a mesh hit at
// t <= stop = min t (>= 0) over the analytic objects after the mesh, every
// later comparison is decided, so the lane stops searching for a closer face.
// LISTS (k_render_px64): the mesh's faces come from the binned lists
// (mesh_lists; pix: the camera ray's pixel, -1 otherwise; light: the shadow
// ray's light, -1 otherwise), and a mesh that no_mesh rules out is skipped
// before its gate (it could only answer "miss": t = -inf or +inf, no update).
// cache (LISTS, or nullptr): kCache* above; cam0: o is the camera origin
// (a camera ray); light >= 0 with the cache: d is that distant light's
// shadow direction.
template <class R, bool COUNT, bool LISTS = false>
__device__ __forceinline__ Hit<R> trace(const RT_CONST RenderParams<R>& p, V3<R> o, V3<R> d, R t_near,
                                        bool active, bool shadow, WaveStats& ws, bool no_mesh = false,
                                        int pix = -1, unsigned pinfo = kPixCount, int light = -1,
                                        const R* cache = nullptr, bool cam0 = false) {
  Hit<R> h{-1, -1, t_near};
  ws.v[STAT_TESTS] += popc32(ballot(active)) * (unsigned int)p.nobj;
  const bool early = shadow && p.shadow_mesh >= 0;
  const bool cached_o = LISTS && cache && cam0;
  const bool cached_d = LISTS && cache && light >= 0;
  // object i's view of the ray (to_object), from the cache where it holds it
  // (returned by value and assembled from local vectors: filled through a
  // reference, field by field, the ray lived in scratch memory — 56 B per
  // lane, ~0.6 GB of write-backs per C3 frame)
  auto obj_ray = [&](int i, const RT_CONST DevObject<R>& ob) -> ORay<R> {
    V3<R> ro, rd, ri{R(0), R(0), R(0)};
    if (cached_o) {
      const R* c = cache + kCacheCamO + 4 * i;
      ro = V3<R>{c[0], c[1], c[2]};
    } else {
      ro = xform_xf<R, true>(ob.xf, ob.w2o, o);
    }
    if (cached_d) {
      const R* c = cache + kCacheLightD + 8 * (light * kCacheObj + i);
      rd = V3<R>{c[0], c[1], c[2]};
      ri = V3<R>{c[4], c[5], c[6]};
    } else {
      rd = xform_xf<R, false>(ob.xf, ob.w2o, d);
    }
    return ORay<R>{ro, rd, ri};
  };
  R stop = -pinf<R>();
  R t_next = R(0);  // LISTS: the t of the object right after the mesh (the same t the main loop would form)
  if (early) {
    stop = pinf<R>();
    for (int i = p.shadow_mesh + 1; i < p.nobj; ++i) {
      const RT_CONST DevObject<R>& ob = cptr(p.objects)[i];
      ORay<R> r;
      if constexpr (LISTS) {
        r = obj_ray(i, ob);
      } else {
        to_object<R>(ob, o, d, r.o, r.d);
      }
      const R t = analytic_t<R>(ob, ob.type, r);
      if (LISTS && i == p.shadow_mesh + 1) t_next = t;
      if (t >= R(0) && t < stop) stop = t;
    }
  }
  for (int i = 0; i < p.nobj; ++i) {
    const RT_CONST DevObject<R>& ob = cptr(p.objects)[i];
    const int type = ob.type;
    ORay<R> r;
    R t;
    int tri = -1;
    if (LISTS && early && i == p.shadow_mesh + 1) {
      t = t_next;
    } else if (LISTS && type == GEOM_MESH && no_mesh) {
      t = -pinf<R>();
    } else if (type != GEOM_MESH) {
      if constexpr (LISTS) {
        r = obj_ray(i, ob);
      } else {
        to_object<R>(ob, o, d, r.o, r.d);
      }
      t = analytic_t<R>(ob, type, r);
    } else {
      V3<R> rd;
      if constexpr (LISTS) {
        r = obj_ray(i, ob);
        rd = r.d;
        if (!cached_d) r.inv = V3<R>{Prec<R>::rcp(rd.x), Prec<R>::rcp(rd.y), Prec<R>::rcp(rd.z)};
      } else {
        to_object<R>(ob, o, d, r.o, rd);
        r.d = rd;
        r.inv = V3<R>{Prec<R>::rcp(rd.x), Prec<R>::rcp(rd.y), Prec<R>::rcp(rd.z)};
      }
      const RT_CONST DevMesh<R>& m = cptr(p.meshes)[ob.mesh];
      // TriangleMesh.intersect (geom.nim:339-358): AABB gate (tmin < 0 ->
      // miss, so rays starting inside the box miss), then closest face.
      const R gate = aabb_ref<R>(V3<R>{m.lo[0], m.lo[1], m.lo[2]}, V3<R>{m.hi[0], m.hi[1], m.hi[2]}, r);
      // no_mesh: the pixel's record proves that no face of the mesh can be
      // hit by this ray: the traversal would find none (best stays -1)
      const bool in = active && gate >= R(0) && !no_mesh;
      R tb = h.t;
      int best = -1;
      if constexpr (LISTS) {
        if (ballot(in) != 0ull && m.root >= 0)
          mesh_lists<R, COUNT>(p, m.root, r, in, early && i == p.shadow_mesh, stop, pix, pinfo, light, tb, best, ws);
      } else {
        traverse<R, COUNT>(p, m.root, r.o, r.d, in, early && i == p.shadow_mesh, stop, tb, best, ws);
      }
      t = !(gate >= R(0)) ? -pinf<R>() : (best >= 0 ? tb : pinf<R>());
      tri = best;
    }
    const bool upd = active && t >= R(0) && t < h.t;
    ws.v[STAT_HITS] += popc32(ballot(upd));
    if (upd) {
      h.t = t;
      h.obj = i;
      h.tri = tri;
    }
  }
  return h;
}

// ---- shade (renderer.nim:71-127) -------------------------------------------
// normal(*) (geom.nim:361-379) for analytic geometry in object space.
template <class R>
__device__ __forceinline__ V3<R> object_normal(const RT_CONST DevObject<R>& ob, int type, V3<R> ho) {
  if (type == GEOM_SPHERE) return normalize_dir<R>(ho);            // geom.nim:364-365
  if (type == GEOM_PLANE) return V3<R>{R(0), R(1), R(0)};          // geom.nim:367-368
  if (type == GEOM_BOX) {                                          // geom.nim:370-379
    const V3<R> vmin{ob.prm[0], ob.prm[1], ob.prm[2]}, vmax{ob.prm[4], ob.prm[5], ob.prm[6]};
    const V3<R> c{(vmin.x + vmax.x) * R(0.5), (vmin.y + vmax.y) * R(0.5), (vmin.z + vmax.z) * R(0.5)};
    const V3<R> pp{ho.x - c.x, ho.y - c.y, ho.z - c.z};
    const V3<R> dd{(vmin.x - vmax.x) * R(0.5), (vmin.y - vmax.y) * R(0.5), (vmin.z - vmax.z) * R(0.5)};
    // float64: the reference's 1.000001 verbatim. float32: the hit point is
    // only good to ~1e-5 of the box size, so 1.000001 can truncate every
    // axis to 0 (a NaN normal); widen to 1.0001 and fall back to the
    // dominant axis.
    const R bias = Prec<R>::exact ? R(1.000001) : R(1.0001);
    const R qx = Prec<R>::div(pp.x, fabs(dd.x)), qy = Prec<R>::div(pp.y, fabs(dd.y)),
            qz = Prec<R>::div(pp.z, fabs(dd.z));
    V3<R> n{R((long long)(qx * bias)), R((long long)(qy * bias)), R((long long)(qz * bias))};
    if constexpr (!Prec<R>::exact) {
      if (n.x == R(0) && n.y == R(0) && n.z == R(0)) {
        const R ax = fabs(qx), ay = fabs(qy), az = fabs(qz);
        if (ax >= ay && ax >= az) n.x = qx < R(0) ? R(-1) : R(1);
        else if (ay >= az) n.y = qy < R(0) ? R(-1) : R(1);
        else n.z = qz < R(0) ? R(-1) : R(1);
      }
    }
    return normalize_dir<R>(n);
  }
  return V3<R>{R(0), R(0), R(0)};
}

// One camera sample: trace + shade with the reflection recursion unrolled
// into a loop of levels. Returns the sample colour (renderer.nim:71-127).
// LEVELS: the reflection levels compiled in (1: a scene without reflective
// materials — no level can follow the camera hit; shade's recursion needs
// depth <= maxRayDepth AND reflection > 0, renderer.nim:104).
template <class R, bool COUNT, bool LISTS = false, int LEVELS = kMaxShadeLevels>
__device__ __forceinline__ V3<R> shade_path(const RT_CONST RenderParams<R>& p, V3<R> o, V3<R> d, bool active,
                                            WaveStats& ws, unsigned pinfo = kPixCount, int pix = -1,
                                            const R* cache = nullptr) {
  constexpr R kPi = R(3.14159265358979323846);
  bool act = active;
  int depth = 1;
  V3<R> terminal{R(0), R(0), R(0)};
  // perf mode: forward weights; exact mode: the reference's nesting order
  // (1 - r)*L + r*inner folded from the innermost level outwards.
  V3<R> facc{R(0), R(0), R(0)};
  R fw = R(1);
  constexpr int kLv = LEVELS > 1 ? LEVELS : 1;
  V3<R> lvl_c[Prec<R>::exact ? kLv : 1];
  R lvl_r[Prec<R>::exact ? kLv : 1];
  int nlev = 0;
  for (int lev = 0; lev < LEVELS; ++lev) {
    if (ballot(act) == 0ull) break;
    // the pixel's record (camera level only): an empty camera-ray list, and
    // per distant light a skip bit for the shadow rays from its camera hits
    const bool cam_skip = lev == 0 && (pinfo & kPixCount) == 0u;
    const Hit<R> hit = trace<R, COUNT, LISTS>(p, o, d, pinf<R>(), act, false, ws, cam_skip, lev == 0 ? pix : -1, pinfo,
                                              -1, cache, lev == 0);
    if (act && hit.obj < 0) terminal = V3<R>{p.bg[0], p.bg[1], p.bg[2]};
    const bool lit = act && hit.obj >= 0;
    const V3<R> hw{o.x + d.x * hit.t, o.y + d.y * hit.t, o.z + d.z * hit.t};
    // Gather the per-object shading inputs with one wave-uniform pass per
    // distinct object hit by the wave (usually one), so the object record is
    // read with scalar loads.
    V3<R> N{R(0), R(0), R(0)};
    V3<R> alb{R(0), R(0), R(0)};
    R refl = R(0);
    unsigned long long pending = ballot(lit);
    while (pending) {
      const int lead = (int)__builtin_ctzll(pending);
      const int oi = __builtin_amdgcn_readlane(hit.obj, lead);
      const bool mine = lit && hit.obj == oi;
      pending &= ~ballot(mine);
      const RT_CONST DevObject<R>& ob = cptr(p.objects)[oi];
      if (mine) {
        V3<R> nrm;
        if (LISTS && cache && hit.tri < 0 && ob.type == GEOM_PLANE) {
          // a plane's normal does not depend on the hit point: its cached N
          const R* c = cache + kCachePlaneN + 4 * oi;
          N = V3<R>{c[0], c[1], c[2]};
          alb = Prec<R>::exact ? V3<R>{ob.albp[0], ob.albp[1], ob.albp[2]} : V3<R>{ob.albedo[0], ob.albedo[1], ob.albedo[2]};
          refl = ob.albedo[3];
          continue;
        }
        if (hit.tri >= 0) {
          const R* fn = p.normals + 3 * (size_t)(cptr(p.meshes)[ob.mesh].normal_base + hit.tri);
          nrm = V3<R>{fn[0], fn[1], fn[2]};
        } else {
          V3<R> ho;
          if constexpr (!Prec<R>::exact) {
            V3<R> dummy;
            to_object<R>(ob, hw, V3<R>{R(0), R(0), R(0)}, ho, dummy);
          } else {
            ho = xform_xf<R, true>(ob.xf, ob.w2o, hw);
          }
          nrm = object_normal<R>(ob, ob.type, ho);
        }
        if constexpr (!Prec<R>::exact) {
          N = ob.xf == XF_GENERAL ? xform<R>(ob.o2w, nrm, R(0)) : nrm;
        } else {
          N = xform_xf<R, false>(ob.xf, ob.o2w, nrm);
        }
        // exact mode: albedo / PI as the host formed it (DevObject.albp, the
        // same IEEE quotient); float mode divides as before
        alb = Prec<R>::exact ? V3<R>{ob.albp[0], ob.albp[1], ob.albp[2]} : V3<R>{ob.albedo[0], ob.albedo[1], ob.albedo[2]};
        refl = ob.albedo[3];
      }
    }
    V3<R> local{R(0), R(0), R(0)};
    for (int li = 0; li < p.nlight; ++li) {
      const RT_CONST DevLight<R>& L = cptr(p.lights)[li];
      V3<R> ldir;
      V3<R> I;
      R dist;
      if (L.type == LIGHT_POINT) {  // light.nim:52-62
        const V3<R> lv{hw.x - L.v[0], hw.y - L.v[1], hw.z - L.v[2]};
        const R r2 = dot4(lv, R(0), lv, R(0));
        ldir = normalize_dir<R>(lv);
        const R den = R(4) * kPi * r2;
        I = V3<R>{Prec<R>::div(L.ci[0], den), Prec<R>::div(L.ci[1], den), Prec<R>::div(L.ci[2], den)};
        dist = Prec<R>::sqrt(r2);
      } else {  // light.nim:46-50
        ldir = V3<R>{L.v[0], L.v[1], L.v[2]};
        I = V3<R>{L.ci[0], L.ci[1], L.ci[2]};
        dist = pinf<R>();
      }
      const V3<R> sd{ldir.x * R(-1), ldir.y * R(-1), ldir.z * R(-1)};
      const V3<R> so{hw.x + N.x * p.bias, hw.y + N.y * p.bias, hw.z + N.z * p.bias};
      ws.v[STAT_SHADOW] += popc32(ballot(lit));
      const bool sh_skip = cam_skip && li < 8 && L.type != LIGHT_POINT && ((pinfo >> (24 + li)) & 1u) != 0u;
      const Hit<R> sh = trace<R, COUNT, LISTS>(p, so, sd, dist, lit, true, ws, sh_skip, -1, kPixCount,
                                               L.type == LIGHT_POINT ? -1 : li, li < kCacheLight ? cache : nullptr);
      if (lit && sh.obj < 0) {  // shadeDiffuse (shader.nim:12-17)
        const R ndl = nmax(R(0), dot4(N, R(0), sd, R(0) * R(-1)));
        const V3<R> ap = Prec<R>::exact ? alb : V3<R>{Prec<R>::div(alb.x, kPi), Prec<R>::div(alb.y, kPi), Prec<R>::div(alb.z, kPi)};
        local.x = local.x + ap.x * I.x * ndl;
        local.y = local.y + ap.y * I.y * ndl;
        local.z = local.z + ap.z * I.z * ndl;
      }
    }
    const bool reflect = lit && refl > R(0) && depth <= p.max_depth;
    if (lit && !reflect) terminal = local;
    if constexpr (Prec<R>::exact) {
      if (reflect) {
        // shift-register push (static indices keep it in registers)
#pragma unroll
        for (int k = kLv - 1; k > 0; --k) {
          lvl_c[k] = lvl_c[k - 1];
          lvl_r[k] = lvl_r[k - 1];
        }
        lvl_c[0] = local;
        lvl_r[0] = refl;
        ++nlev;
      }
    } else {
      if (reflect) {
        const R wl = fw * (R(1) - refl);
        facc = V3<R>{facc.x + wl * local.x, facc.y + wl * local.y, facc.z + wl * local.z};
        fw = fw * refl;
      }
    }
    ws.v[STAT_REFL] += popc32(ballot(reflect));
    if (reflect) {
      // renderer.nim:109-118
      const R ndi = R(2) * dot4(N, R(0), d, R(0));
      const V3<R> rd{d.x - N.x * ndi, d.y - N.y * ndi, d.z - N.z * ndi};
      o = V3<R>{hw.x + rd.x * p.bias, hw.y + rd.y * p.bias, hw.z + rd.z * p.bias};
      d = rd;
      ++depth;
    }
    act = reflect;
  }
  if constexpr (Prec<R>::exact) {
    V3<R> c = terminal;
#pragma unroll
    for (int k = 0; k < kLv; ++k) {
      if (k < nlev) {
        const R r = lvl_r[k];
        c = V3<R>{(R(1) - r) * lvl_c[k].x + r * c.x, (R(1) - r) * lvl_c[k].y + r * c.y,
                  (R(1) - r) * lvl_c[k].z + r * c.z};
      }
    }
    return c;
  } else {
    (void)lvl_c;
    (void)lvl_r;
    (void)nlev;
    return V3<R>{facc.x + fw * terminal.x, facc.y + fw * terminal.y, facc.z + fw * terminal.z};
  }
}

// One camera sample of a LEAN pixel in k_render_px64 (RenderParams.lean_plane
// >= 0: one mesh + one non-reflective plane, distant lights only): the
// pixel's record says its camera rays miss the mesh (empty list) and so do
// its shadow rays to every light (skip bits), so shade_path<double, ...,
// LISTS> would test the mesh nowhere (t = -inf, no update) and this is the
// rest of it — the same operations in the same order on the plane alone:
// trace (renderer.nim:47-67) counts nobj tests per ray and the plane's hits,
// shade (renderer.nim:71-104) adds shadeDiffuse per unshadowed light. The
// sample-invariant values come from the block cache: the plane's view of the
// camera origin and of each shadow direction, its normal, and each light's
// shading term (kCacheLeanTerm: albp * ci * ndl with the same rounding as
// the per-sample product). The compiler keeps only the y components the
// plane test reads (plane_ref), which is what makes this path cheap.
__device__ __forceinline__ V3<double> px64_lean_sample(const RT_CONST RenderParams<double>& p, V3<double> o,
                                                       V3<double> d, bool active, WaveStats& ws,
                                                       const double* cache) {
  using R = double;
  const int pl = p.lean_plane;
  const RT_CONST DevObject<R>& ob = cptr(p.objects)[pl];
  const int xf = ob.xf;
  const unsigned nobj = (unsigned)p.nobj;
  ws.v[STAT_TESTS] += popc32(ballot(active)) * nobj;
  const R* co = cache + kCacheCamO + 4 * pl;
  ORay<R> r;
  r.o = V3<R>{co[0], co[1], co[2]};
  r.d = xform_xf<R, false>(xf, ob.w2o, d);
  r.inv = V3<R>{R(0), R(0), R(0)};
  const R t = plane_ref<R>(r);
  const bool lit = active && t >= R(0) && t < pinf<R>();
  ws.v[STAT_HITS] += popc32(ballot(lit));
  V3<R> terminal{R(0), R(0), R(0)};
  if (active && !lit) terminal = V3<R>{p.bg[0], p.bg[1], p.bg[2]};
  const R ht = lit ? t : pinf<R>();  // hit.t (t_near = inf without a hit)
  const V3<R> hw{o.x + d.x * ht, o.y + d.y * ht, o.z + d.z * ht};
  const R* cn = cache + kCachePlaneN + 4 * pl;
  const V3<R> N{cn[0], cn[1], cn[2]};
  const V3<R> so{hw.x + N.x * p.bias, hw.y + N.y * p.bias, hw.z + N.z * p.bias};
  ORay<R> sr;
  sr.o = xform_xf<R, true>(xf, ob.w2o, so);
  const unsigned nlit = popc32(ballot(lit));
  V3<R> local{R(0), R(0), R(0)};
  for (int li = 0; li < p.nlight; ++li) {
    ws.v[STAT_SHADOW] += nlit;
    ws.v[STAT_TESTS] += nlit * nobj;
    const R* cd = cache + kCacheLightD + 8 * (li * kCacheObj + pl);
    sr.d = V3<R>{cd[0], cd[1], cd[2]};
    sr.inv = V3<R>{cd[4], cd[5], cd[6]};
    const R ts = plane_ref<R>(sr);
    const bool blocked = lit && ts >= R(0) && ts < pinf<R>();
    ws.v[STAT_HITS] += popc32(ballot(blocked));
    if (lit && !blocked) {
      const R* tm = cache + kCacheLeanTerm + 4 * li;
      local = V3<R>{local.x + tm[0], local.y + tm[1], local.z + tm[2]};
    }
  }
  if (lit) terminal = local;
  return terminal;
}

// Move the wave's 32-bit counters into the per-lane 64-bit totals.
__device__ __forceinline__ void flush_stats(WaveStats& ws, unsigned long long& tot, int lane) {
#pragma unroll
  for (int k = 0; k < kStatSlots; ++k) {
    tot += (lane == k) ? (unsigned long long)ws.v[k] : 0ull;
    ws.v[k] = 0u;
  }
}

// ---- the render kernel -----------------------------------------------------
#ifndef RTMI_MIN_WAVES
#define RTMI_MIN_WAVES 1
#endif
template <class R, bool COUNT>
__global__ __launch_bounds__(256, RTMI_MIN_WAVES) void k_render(const RenderParams<R> params_by_value) {
  (void)params_by_value;  // read through rparams()
  const RT_CONST RenderParams<R>& p = rparams<R>();
  const int lane = (int)__lane_id();
  const long long wave = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const long long nwaves = (long long)gridDim.x * (blockDim.x >> 6);
  const int L = p.lanes_per_px;
  const int sub = lane % L;
  const int pix = lane / L;
  const int tpx = pix % p.tile_x, tpy = pix / p.tile_x;
  const int iters = (p.spp + L - 1) / L;
  const bool grid_aa = p.aa_kind != 0;
  WaveStats ws;
#pragma unroll
  for (int k = 0; k < kStatSlots; ++k) ws.v[k] = 0u;
  unsigned long long tot = 0ull;

  for (long long g = wave; g < p.ngroups; g += nwaves) {
    const int gx = (int)(g % p.tiles_x), gy = (int)(g / p.tiles_x);
    const int j = gx * p.tile_x + tpx;
    const int k = gy * p.tile_y + tpy;
    const int x = j * p.step;
    int y, out_row;
    bool valid = j < p.ncols && k < p.nrows;
    if (p.mode == 0) {
      y = p.y0 + k * p.step;
      out_row = y;
    } else {
      const int lb = k / p.band_h, rr = k % p.band_h;
      y = (lb * p.world + p.rank) * p.band_h + rr;
      out_row = k;
      valid = valid && y < p.height;
    }
    if (p.step < p.max_step) {  // progressive refinement skip (renderer.nim:175-178)
      const int mask = p.step * 2 - 1;
      if ((x & mask) == 0 && (y & mask) == 0) valid = false;
    }
    V3<R> acc{R(0), R(0), R(0)};
    const unsigned pinfo = (!COUNT && p.pix_info && valid) ? p.pix_info[(size_t)y * p.width + x] : kPixCount;
    // stochastic kinds (sampling.nim:21-113): this lane's pixel table, built
    // sequentially like calcPixel's `samples` in its slice of the scratch
    R* tsx = nullptr;
    R* tsy = nullptr;
    if (p.aa_kind >= 2 && valid) {
      tsx = p.sample_scratch + (size_t)(wave * 64 + lane) * 2 * (size_t)p.spp;
      tsy = tsx + p.spp;
      sample_table_seq<R>(p.aa_kind, p.grid_m, rng_pixel_key(p.seed, x, y), tsx, tsy);
    }
    for (int it = 0; it < iters; ++it) {
      const int s = it * L + sub;
      const bool sv = valid && s < p.spp;
      R px = R(x), py = R(y);
      if (tsx) {
        px = R(x) + tsx[s];
        py = R(y) + tsy[s];
      } else if (grid_aa) {  // grid() sampling.nim:5-18, p[j*m + i]
        const int si = s % p.grid_m, sj = s / p.grid_m;
        px = R(x) + (R(si) * p.sample_step + p.sample_off);
        py = R(y) + (R(sj) * p.sample_step + p.sample_off);
      }
      // castPrimaryRay (renderer.nim:31-44)
      const R cx = (Prec<R>::div(R(2) * px * p.aspect, R(p.width)) - p.aspect) * p.f;
      const R cy = (R(1) - Prec<R>::div(R(2) * py, R(p.height))) * p.f;
      const V3<R> dn = normalize_dir<R>(V3<R>{cx, cy, R(-1)});
      const V3<R> o = xform<R>(p.c2w, V3<R>{R(0), R(0), R(0)}, R(1));
      const V3<R> d = xform<R>(p.c2w, dn, R(0));
      ws.v[STAT_PRIMARY] += popc32(ballot(sv));
      const V3<R> c = shade_path<R, COUNT>(p, o, d, sv, ws, pinfo);
      if (sv) {
        if (grid_aa) {
          acc = V3<R>{acc.x + c.x, acc.y + c.y, acc.z + c.z};
        } else {
          acc = c;
        }
      }
      if ((it & 63) == 63) flush_stats(ws, tot, lane);
    }
    flush_stats(ws, tot, lane);
    // sum the L lanes of each pixel (exact mode launches with L = 1)
    for (int off = 1; off < L; off <<= 1) {
      acc.x += __shfl_xor(acc.x, off);
      acc.y += __shfl_xor(acc.y, off);
      acc.z += __shfl_xor(acc.z, off);
    }
    if (valid && sub == 0) {
      if (grid_aa) acc = V3<R>{acc.x * p.inv_len, acc.y * p.inv_len, acc.z * p.inv_len};
      const float cr = (float)acc.x, cg = (float)acc.y, cb = (float)acc.z;
      if (p.mode == 0 && p.step > 1) {
        const int xe = min(x + p.step, p.width), ye = min(y + p.step, p.height);
        for (int yy = y; yy < ye; ++yy)
          for (int xx = x; xx < xe; ++xx) {
            float* q = p.fb + ((size_t)yy * p.width + xx) * 3;
            q[0] = cr; q[1] = cg; q[2] = cb;
          }
      } else {
        float* q = p.fb + ((size_t)out_row * p.width + x) * 3;
        q[0] = cr; q[1] = cg; q[2] = cb;
      }
    }
  }
  if (lane < kStatSlots) p.partials[wave * kStatSlots + lane] = tot;
}

// ---- k_render_px64: float64, one pixel per wave -----------------------------
// The parity mode's fast layout for akGrid with >= 64 samples per pixel: a
// wave's 64 lanes trace 64 samples of ONE pixel (s = 64 it + lane), so every
// ray of a step shares the pixel's camera-ray face list, and its shadow rays
// a few light-grid cells (mesh_lists) — the same answers as the per-ray BVH,
// in the reference's float64 arithmetic.
//
// calcPixel (renderer.nim:149-159) sums the samples in sample order; to keep
// that sum bit for bit a wave renders P pixels at a time: step `it` of each
// pixel j leaves its 64 sample colours in the wave's LDS row j, then lane j
// adds row j's colours to pixel j's running sum in sample order (64
// dependent adds, P chains side by side) before the next step overwrites
// the rows. Rows are padded to 65 doubles so the summing lanes' reads fall
// in different banks.
// (the reflective instantiation — LEVELS > 1, shade_path's per-level state
// — runs at 2 waves per SIMD: at 3 it spilled 71 VGPRs, 336 B per lane)
#ifndef RTMI_PX64_WAVES
#define RTMI_PX64_WAVES 3
#endif
template <int P, int LEVELS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LEVELS > 1 ? 2 : RTMI_PX64_WAVES))) void k_render_px64(const RenderParams<double> params_by_value) {
  using R = double;
  (void)params_by_value;  // read through rparams()
  const RT_CONST RenderParams<R>& p = rparams<R>();
  constexpr int kRow = 66;  // 16-B aligned rows; row stride 4 banks apart: the 3P summing lanes' reads never conflict
  __shared__ __attribute__((aligned(16))) double sbuf[4][P * 3 * kRow];
  const int lane = (int)__lane_id();
  const int wib = (int)(threadIdx.x >> 6);
  double* buf = sbuf[wib];
  const long long wave = (long long)blockIdx.x * (blockDim.x >> 6) + wib;
  const long long nwaves = (long long)gridDim.x * (blockDim.x >> 6);
  const int iters = (p.spp + 63) / 64;
  const long long npx = (long long)p.nrows * p.ncols;
  const long long nbatch = (npx + P - 1) / P;
  WaveStats ws;
#pragma unroll
  for (int k = 0; k < kStatSlots; ++k) ws.v[k] = 0u;
  unsigned long long tot = 0ull;
  // the camera origin (castPrimaryRay: cameraToWorld * (0, 0, 0, 1)) is the
  // same for every sample
  const V3<R> o = xform<R>(p.c2w, V3<R>{R(0), R(0), R(0)}, R(1));
  // the block's cache (kCache*): per object its view of the camera origin and,
  // for a plane, its world normal; per distant light the shadow direction in
  // each object's space and its reciprocals — the very operations trace() and
  // shade_path() would apply per sample
  __shared__ double cache[kCacheDoubles];
  const bool use_cache = p.nobj <= kCacheObj && p.nlight <= kCacheLight;
  if (use_cache) {
    const int nobj = p.nobj;
    for (int t = (int)threadIdx.x; t < nobj * (1 + p.nlight); t += (int)blockDim.x) {
      const int i = t % nobj, l = t / nobj - 1;
      const RT_CONST DevObject<R>& ob = cptr(p.objects)[i];
      if (l < 0) {
        const V3<R> ro = xform_xf<R, true>(ob.xf, ob.w2o, o);
        double* c = cache + kCacheCamO + 4 * i;
        c[0] = ro.x; c[1] = ro.y; c[2] = ro.z;
        const V3<R> n = xform_xf<R, false>(ob.xf, ob.o2w, V3<R>{R(0), R(1), R(0)});  // geom.nim:367-368, renderer.nim:88
        double* cn = cache + kCachePlaneN + 4 * i;
        cn[0] = n.x; cn[1] = n.y; cn[2] = n.z;
      } else {
        const RT_CONST DevLight<R>& L = cptr(p.lights)[l];
        const V3<R> sd{R(L.v[0]) * R(-1), R(L.v[1]) * R(-1), R(L.v[2]) * R(-1)};  // shade: -lightDir
        const V3<R> rd = xform_xf<R, false>(ob.xf, ob.w2o, sd);
        double* c = cache + kCacheLightD + 8 * (l * kCacheObj + i);
        c[0] = rd.x; c[1] = rd.y; c[2] = rd.z;
        c[4] = Prec<R>::rcp(rd.x); c[5] = Prec<R>::rcp(rd.y); c[6] = Prec<R>::rcp(rd.z);
      }
    }
    __syncthreads();
    // the lean plane's per-light shading terms (shade_path's product, same
    // operands: the cached normal, -lightDir, albedo / PI, color * intensity)
    if (p.lean_plane >= 0 && (int)threadIdx.x < p.nlight) {
      const int l = (int)threadIdx.x;
      const RT_CONST DevObject<R>& ob = cptr(p.objects)[p.lean_plane];
      const RT_CONST DevLight<R>& L = cptr(p.lights)[l];
      const double* cn = cache + kCachePlaneN + 4 * p.lean_plane;
      const V3<R> N{cn[0], cn[1], cn[2]};
      const V3<R> ldir{L.v[0], L.v[1], L.v[2]};
      const V3<R> sd{ldir.x * R(-1), ldir.y * R(-1), ldir.z * R(-1)};
      const V3<R> I{L.ci[0], L.ci[1], L.ci[2]};
      const R ndl = nmax(R(0), dot4(N, R(0), sd, R(0) * R(-1)));
      double* tm = cache + kCacheLeanTerm + 4 * l;
      tm[0] = ob.albp[0] * I.x * ndl;
      tm[1] = ob.albp[1] * I.y * ndl;
      tm[2] = ob.albp[2] * I.z * ndl;
    }
    __syncthreads();
  }
  const double* cch = use_cache ? cache : nullptr;
  // a lean pixel: empty camera-ray list and every light's skip bit set
  // (the reflective instantiation keeps the general path only: it runs at 2
  // waves per SIMD on its register budget)
  const unsigned lean_need = LEVELS == 1 && use_cache && p.lean_plane >= 0 ? ((1u << p.nlight) - 1u) << 24 : 0u;

  // pixel g of the launch: image (x, y), its output row, whether it renders
  auto pixel_of = [&](long long g, int& x, int& y, int& out_row) -> bool {
    const int k = (int)(g / p.ncols), j = (int)(g % p.ncols);
    x = j * p.step;
    bool valid = g < npx;
    if (p.mode == 0) {
      y = p.y0 + k * p.step;
      out_row = y;
    } else {
      const int lb = k / p.band_h, rr = k % p.band_h;
      y = (lb * p.world + p.rank) * p.band_h + rr;
      out_row = k;
      valid = valid && y < p.height;
    }
    if (p.step < p.max_step) {  // progressive refinement skip (renderer.nim:175-178)
      const int mask = p.step * 2 - 1;
      if ((x & mask) == 0 && (y & mask) == 0) valid = false;
    }
    return valid;
  };

  for (long long b = wave; b < nbatch; b += nwaves) {
    // the batch's pixels, pixel j in lane j < P (its image position, output
    // row and record), read back by readlane: one pixel_of per pixel and
    // batch instead of one per pixel and step
    int bx = 0, by = 0, brow = 0;
    unsigned binfo = kPixCount;
    bool bok = false;
    if (lane < P) {
      bok = pixel_of(b * P + lane, bx, by, brow);
      if (bok && p.pix_info) binfo = p.pix_info[by * p.width + bx];
    }
    const unsigned long long okm = ballot(bok);
    // lane 3j + c < 3P: component c of pixel j's running sum (sample order)
    R acc = R(0);
    for (int it = 0; it < iters; ++it) {
      const int s = it * 64 + lane;
      const bool sv = s < p.spp;
      const int si = s % p.grid_m, sj = s / p.grid_m;
      // castPrimaryRay's y term depends on the row and the sample only: the
      // batch's pixels usually share a row, so it is formed once per row
      int cy_row = -1;
      R cy = R(0);
      for (int j = 0; j < P; ++j) {
        if (!((okm >> j) & 1ull)) continue;
        const int x = __builtin_amdgcn_readlane(bx, j), y = __builtin_amdgcn_readlane(by, j);
        const unsigned pinfo = (unsigned)__builtin_amdgcn_readlane((int)binfo, j);
        const int pix = y * p.width + x;
        // grid() sampling.nim:5-18, p[j*m + i]; castPrimaryRay (renderer.nim:31-44)
        const R px = R(x) + (R(si) * p.sample_step + p.sample_off);
        if (y != cy_row) {
          const R py = R(y) + (R(sj) * p.sample_step + p.sample_off);
          cy = (R(1) - Prec<R>::div(R(2) * py, R(p.height))) * p.f;
          cy_row = y;
        }
        const R cx = (Prec<R>::div(R(2) * px * p.aspect, R(p.width)) - p.aspect) * p.f;
        const V3<R> dn = normalize_dir<R>(V3<R>{cx, cy, R(-1)});
        const V3<R> d = xform<R>(p.c2w, dn, R(0));
        ws.v[STAT_PRIMARY] += popc32(ballot(sv));
        V3<R> c;
        const bool lean_px = lean_need != 0u && (pinfo & (kPixCount | lean_need)) == lean_need;
#if defined(RTMI_DIAG) && defined(RTMI_PX64_ONLY)
        // diagnostic builds (tools/build_variant.sh): 1 = lean samples only,
        // 2 = general samples only — a time split, wrong images on purpose
        if (lean_px != (RTMI_PX64_ONLY == 1)) {
          c = V3<R>{R(0), R(0), R(0)};
        } else
#endif
        if (lean_px)
          c = px64_lean_sample(rparams<R>(), o, d, sv, ws, cch);
        else
          c = shade_path<R, false, true, LEVELS>(rparams<R>(), o, d, sv, ws, pinfo, pix, cch);
        buf[(j * 3 + 0) * kRow + lane] = c.x;
        buf[(j * 3 + 1) * kRow + lane] = c.y;
        buf[(j * 3 + 2) * kRow + lane] = c.z;
      }
      // the rows are read by other lanes of this wave: LDS operations of one
      // wave complete in order, the barrier keeps the compiler from moving
      // the reads above the writes
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // calcPixel's sum (renderer.nim:149-159), each of the 3P chains in its
      // own lane, in sample order; a full step reads its row two samples per
      // 128-bit LDS read (rows of pixels skipped this batch are never used)
      if (lane < 3 * P) {
        const double* row = buf + lane * kRow;
        const int nv = min(64, p.spp - it * 64);
        if (nv == 64) {
          const double2* r2 = (const double2*)row;
#pragma unroll 8
          for (int k = 0; k < 32; ++k) {
            const double2 v = r2[k];
            acc = acc + v.x;
            acc = acc + v.y;
          }
        } else {
          for (int k = 0; k < nv; ++k) acc = acc + row[k];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // empty the 32-bit wave counters every 16 steps, as k_render does every
      // 64 samples: STAT_TESTS grows by 64 x nobj per trace, P pixels x
      // (1 + lights) x levels traces per step
      if ((it & 15) == 15) flush_stats(ws, tot, lane);
    }
    flush_stats(ws, tot, lane);
    // pixel j's three sums to lane j
    const R ax = __shfl(acc, 3 * lane + 0), ay = __shfl(acc, 3 * lane + 1), az = __shfl(acc, 3 * lane + 2);
    if (bok) {  // lanes j < P
      const int x = bx, y = by, out_row = brow;
      const float cr = (float)(ax * p.inv_len), cg = (float)(ay * p.inv_len), cb = (float)(az * p.inv_len);
      if (p.mode == 0 && p.step > 1) {
        const int xe = min(x + p.step, p.width), ye = min(y + p.step, p.height);
        for (int yy = y; yy < ye; ++yy)
          for (int xx = x; xx < xe; ++xx) {
            float* q = p.fb + ((size_t)yy * p.width + xx) * 3;
            q[0] = cr; q[1] = cg; q[2] = cb;
          }
      } else {
        float* q = p.fb + ((size_t)out_row * p.width + x) * 3;
        q[0] = cr; q[1] = cg; q[2] = cb;
      }
    }
  }
  if (lane < kStatSlots) p.partials[wave * kStatSlots + lane] = tot;
}

}  // namespace rtmi
