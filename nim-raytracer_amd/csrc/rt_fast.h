// rt_fast.h — the float32 performance kernel (RT_FP32).
//
// Same algorithm and Stats semantics as the float64 parity kernel
// (rt_device.h: trace = linear closest hit over the scene's objects,
// renderer.nim:47-67; shade with one shadow ray per light and the reflection
// recursion, renderer.nim:71-127), restructured for the gfx950 instruction
// stream:
//  * compact 64-byte object records read with ONE scalar load each
//    (s_load_dwordx16), identity / translation transforms short-circuited;
//  * camera constants precomputed on the host: a primary ray is two FMAs,
//    one v_rsq and a 3x3 basis combination;
//  * hardware v_rcp / v_rsq / v_sqrt instead of the IEEE division and sqrt
//    expansions; sample indices advanced incrementally (no integer division
//    in the sample loop); ballots through __builtin_amdgcn_ballot_w64 so
//    lane masks stay in SGPRs;
//  * the wave-coherent BVH traversal of rt_device.h (scalar node / triangle
//    fetches, 64-lane VGPR stack, ballot-driven child selection).
#pragma once
#include <hip/hip_runtime.h>

#include "rt_common.h"

#ifndef RT_CONST
#if defined(__HIP_DEVICE_COMPILE__)
#define RT_CONST __attribute__((address_space(4)))  // scalar (constant) loads
#else
#define RT_CONST
#endif
#endif

#ifndef RTMI_BVH4
#define RTMI_BVH4 0
#endif
#ifndef RTMI_LEAF_BATCH
#define RTMI_LEAF_BATCH 0
#endif

namespace rtmi {
namespace fast {

template <class T>
__device__ __forceinline__ const RT_CONST T* cp(const T* p) {
  return (const RT_CONST T*)(p);
}

__device__ __forceinline__ unsigned long long bal(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ unsigned int pc(unsigned long long m) { return (unsigned int)__builtin_popcountll(m); }
__device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float rsq(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float finf() { return __builtin_huge_valf(); }

struct F3 {
  float x, y, z;
};
__device__ __forceinline__ F3 f3(float x, float y, float z) { return F3{x, y, z}; }
__device__ __forceinline__ float dot3(F3 a, F3 b) { return __builtin_fmaf(a.x, b.x, __builtin_fmaf(a.y, b.y, a.z * b.z)); }

struct Stats32 {
  unsigned int v[kStatSlots];
};

#ifdef RTMI_STAMPS
// Diagnostic build only (never the measured kernel): shader-clock stamps
// accumulated into the traversal counter slots 5..8.
__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define RT_STAMP(var) const unsigned long long var = stamp()
#define RT_ACC(slot, a, b) ws.v[slot] += (unsigned int)((b) - (a))
#else
#define RT_STAMP(var)
#define RT_ACC(slot, a, b)
#endif

struct Hit {
  int obj;
  int tri;
  float t;
};

// World -> object space (FObj.xf classification).
__device__ __forceinline__ void to_object(const FastParams& p, const FObj& ob, int i, F3 o, F3 d, F3& ro,
                                          F3& rd) {
  if (ob.xf == XF_IDENTITY) {
    ro = o;
    rd = d;
  } else if (ob.xf == XF_TRANSLATE) {
    ro = f3(o.x + ob.t[0], o.y + ob.t[1], o.z + ob.t[2]);
    rd = d;
  } else {
    const RT_CONST FObjX& x = cp(p.objx)[i];
    const float* m = x.w2o;  // m[c*3 + r], c = 0..3
    ro = f3(__builtin_fmaf(m[0], o.x, __builtin_fmaf(m[3], o.y, __builtin_fmaf(m[6], o.z, m[9]))),
            __builtin_fmaf(m[1], o.x, __builtin_fmaf(m[4], o.y, __builtin_fmaf(m[7], o.z, m[10]))),
            __builtin_fmaf(m[2], o.x, __builtin_fmaf(m[5], o.y, __builtin_fmaf(m[8], o.z, m[11]))));
    rd = f3(__builtin_fmaf(m[0], d.x, __builtin_fmaf(m[3], d.y, m[6] * d.z)),
            __builtin_fmaf(m[1], d.x, __builtin_fmaf(m[4], d.y, m[7] * d.z)),
            __builtin_fmaf(m[2], d.x, __builtin_fmaf(m[5], d.y, m[8] * d.z)));
  }
}

// AABB.intersect (geom.nim:76-96) in IEEE min/max form; -inf = miss.
__device__ __forceinline__ float aabb(const float* lo, const float* hi, F3 o, F3 inv) {
  const float ax = (lo[0] - o.x) * inv.x, bx = (hi[0] - o.x) * inv.x;
  const float ay = (lo[1] - o.y) * inv.y, by = (hi[1] - o.y) * inv.y;
  const float az = (lo[2] - o.z) * inv.z, bz = (hi[2] - o.z) * inv.z;
  const float tmin = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
  const float tmax = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz)) * 1.00000024f;
  return tmin <= tmax ? tmin : -finf();
}

// Sphere.intersect (geom.nim:215-237) incl. the `/ 2*a` precedence.
__device__ __forceinline__ float sphere(float radius, F3 o, F3 d) {
  const float a = dot3(d, d);
  const float b = 2.0f * dot3(d, o);
  const float c = dot3(o, o) - radius * radius;
  const float delta = b * b - 4.0f * a * c;
  const float sb = b > 0.0f ? 1.0f : (b < 0.0f ? -1.0f : 0.0f);
  const float t1 = ((-b - sb * fsqrt(delta)) * 0.5f) * a;
  const float t2 = c * rcp(a * t1);
  const float t = t1 <= t2 ? t1 : t2;
  return delta >= 0.0f ? t : -finf();
}

// Plane.intersect (geom.nim:240-248): y = 0.
__device__ __forceinline__ float plane(F3 o, F3 d) {
  return fabsf(d.y) > 1e-6f ? -o.y * rcp(d.y) : -finf();
}

// rayTriangleIntersectFast (geom.nim:283-336), single-sided.
__device__ __forceinline__ float triangle(const TriF32& tri, F3 o, F3 d) {
  const float e1x = tri.e1[0], e1y = tri.e1[1], e1z = tri.e1[2];
  const float e2x = tri.e2[0], e2y = tri.e2[1], e2z = tri.e2[2];
  const float px = d.y * e2z - d.z * e2y;
  const float py = d.z * e2x - d.x * e2z;
  const float pz = d.x * e2y - d.y * e2x;
  const float det = __builtin_fmaf(e1x, px, __builtin_fmaf(e1y, py, e1z * pz));
  const float inv_det = rcp(det);
  const float tx = o.x - tri.v0[0], ty = o.y - tri.v0[1], tz = o.z - tri.v0[2];
  const float u = __builtin_fmaf(tx, px, __builtin_fmaf(ty, py, tz * pz)) * inv_det;
  const float qx = ty * e1z - tz * e1y;
  const float qy = tz * e1x - tx * e1z;
  const float qz = tx * e1y - ty * e1x;
  const float v = __builtin_fmaf(d.x, qx, __builtin_fmaf(d.y, qy, d.z * qz)) * inv_det;
  const float t = __builtin_fmaf(e2x, qx, __builtin_fmaf(e2y, qy, e2z * qz)) * inv_det;
  const bool ok = det >= 0.000001f && u >= 0.0f && u <= 1.0f && v >= 0.0f && u + v <= 1.0f;
  return ok ? t : -finf();
}

// Leaf: closest/any hit over `n` triangles starting at `first` for lanes `h`.
__device__ __forceinline__ void leaf(const FastParams& p, int first, int n, bool h, F3 o, F3 d, float& tbest,
                                     int& best_id) {
  for (int k = 0; k < n; ++k) {
    const TriF32 tri = cp(p.tris)[first + k];
    const float t = triangle(tri, o, d);
    const int id = tri.id;
    if (h && t >= 0.0f && (t < tbest || (t == tbest && id < best_id))) {
      tbest = t;
      best_id = id;
    }
  }
}

// Wave-coherent closest/any hit over one mesh BVH2 (64-B nodes, both child
// boxes per fetch). Selected with -DRTMI_BVH4=0.
template <bool COUNT>
__device__ __forceinline__ void traverse2(const FastParams& p, int root, F3 o, F3 d, bool active, bool anyhit,
                                          float& tbest, int& best_id, Stats32& ws) {
  if (bal(active) == 0ull) return;
  RT_STAMP(t_enter);
  const float e = 1e-20f;
  const float dx = fabsf(d.x) < e ? __builtin_copysignf(e, d.x) : d.x;
  const float dy = fabsf(d.y) < e ? __builtin_copysignf(e, d.y) : d.y;
  const float dz = fabsf(d.z) < e ? __builtin_copysignf(e, d.z) : d.z;
  const F3 ni = f3(rcp(dx), rcp(dy), rcp(dz));
  const F3 oi = f3(o.x * ni.x, o.y * ni.y, o.z * ni.z);
  const int lane = (int)__lane_id();
  int stack = 0;
  int sp = 0;
  int node = root;
  for (int iter = 0; iter < p.max_iters; ++iter) {
    const BvhNode nd = cp(p.nodes)[node];
    if constexpr (COUNT) {
      ws.v[STAT_NODE_FETCH] += 1u;
      ws.v[STAT_LANE_NODES] += pc(bal(active));
    }
    const float ax0 = __builtin_fmaf(nd.lo0[0], ni.x, -oi.x), bx0 = __builtin_fmaf(nd.hi0[0], ni.x, -oi.x);
    const float ay0 = __builtin_fmaf(nd.lo0[1], ni.y, -oi.y), by0 = __builtin_fmaf(nd.hi0[1], ni.y, -oi.y);
    const float az0 = __builtin_fmaf(nd.lo0[2], ni.z, -oi.z), bz0 = __builtin_fmaf(nd.hi0[2], ni.z, -oi.z);
    const float ax1 = __builtin_fmaf(nd.lo1[0], ni.x, -oi.x), bx1 = __builtin_fmaf(nd.hi1[0], ni.x, -oi.x);
    const float ay1 = __builtin_fmaf(nd.lo1[1], ni.y, -oi.y), by1 = __builtin_fmaf(nd.hi1[1], ni.y, -oi.y);
    const float az1 = __builtin_fmaf(nd.lo1[2], ni.z, -oi.z), bz1 = __builtin_fmaf(nd.hi1[2], ni.z, -oi.z);
    const float tn0 = fmaxf(fmaxf(fminf(ax0, bx0), fminf(ay0, by0)), fmaxf(fminf(az0, bz0), 0.0f));
    const float tf0 = fminf(fminf(fmaxf(ax0, bx0), fmaxf(ay0, by0)), fminf(fmaxf(az0, bz0), tbest));
    const float tn1 = fmaxf(fmaxf(fminf(ax1, bx1), fminf(ay1, by1)), fmaxf(fminf(az1, bz1), 0.0f));
    const float tf1 = fminf(fminf(fmaxf(ax1, bx1), fmaxf(ay1, by1)), fminf(fmaxf(az1, bz1), tbest));
    const bool h0 = active && tn0 <= tf0 * 1.0000004f;
    const bool h1 = active && tn1 <= tf1 * 1.0000004f;
    unsigned long long m0 = (nd.n0 > 0 || nd.c0 >= 0) ? bal(h0) : 0ull;
    unsigned long long m1 = (nd.n1 > 0 || nd.c1 >= 0) ? bal(h1) : 0ull;
    if (nd.n0 > 0 && m0) {
      if constexpr (COUNT) {
        ws.v[STAT_TRI_FETCH] += (unsigned int)nd.n0;
        ws.v[STAT_LANE_TRIS] += pc(m0) * (unsigned int)nd.n0;
      }
      leaf(p, nd.c0, nd.n0, h0, o, d, tbest, best_id);
      if (anyhit) active = active && best_id < 0;
      m0 = 0ull;
    }
    if (nd.n1 > 0 && m1) {
      if constexpr (COUNT) {
        ws.v[STAT_TRI_FETCH] += (unsigned int)nd.n1;
        ws.v[STAT_LANE_TRIS] += pc(m1) * (unsigned int)nd.n1;
      }
      leaf(p, nd.c1, nd.n1, h1, o, d, tbest, best_id);
      if (anyhit) active = active && best_id < 0;
      m1 = 0ull;
    }
    if (anyhit && bal(active) == 0ull) break;
    if (m0 && m1) {
      const unsigned long long near0 = bal(h0 && h1 && tn0 <= tn1);
      const bool first0 = pc(near0) * 2u >= pc(m0 & m1);
      const int near = first0 ? nd.c0 : nd.c1;
      const int far = first0 ? nd.c1 : nd.c0;
      stack = (lane == sp) ? far : stack;
      ++sp;
      node = near;
    } else if (m0) {
      node = nd.c0;
    } else if (m1) {
      node = nd.c1;
    } else {
      if (sp == 0) break;
      --sp;
      node = __builtin_amdgcn_readlane(stack, sp);
    }
  }
#ifdef RTMI_STAMPS
  { RT_STAMP(t_exit); RT_ACC(5, t_enter, t_exit); }
#endif
}

__device__ __forceinline__ void cswap(unsigned& ka, int& ca, unsigned& kb, int& cb) {
  const bool sw = kb < ka;
  const unsigned k = sw ? kb : ka;
  const int c = sw ? cb : ca;
  kb = sw ? ka : kb;
  cb = sw ? ca : cb;
  ka = k;
  ca = c;
}

// Wave-coherent closest/any hit over one mesh's BVH4 (rt_common.h Bvh4Node).
// The node index and the stack are wave-uniform: one 128-B node is fetched
// with scalar loads, every lane tests the four child boxes against its own
// ray (four independent slab tests: ILP), ballots decide which children the
// wave visits, leaves are tested immediately, internal children are ordered
// by the lead lane's entry distance (a scalar sorting network on the float
// bits; entry distances are >= 0) and all but the nearest are pushed onto
// the 64-lane VGPR stack. Must be called from wave-uniform control flow.
template <bool COUNT>
__device__ __forceinline__ void traverse4(const FastParams& p, int root, F3 o, F3 d, bool active, bool anyhit,
                                          float& tbest, int& best_id, Stats32& ws) {
  if (bal(active) == 0ull) return;
  RT_STAMP(t_enter);
  const float e = 1e-20f;
  const float dx = fabsf(d.x) < e ? __builtin_copysignf(e, d.x) : d.x;
  const float dy = fabsf(d.y) < e ? __builtin_copysignf(e, d.y) : d.y;
  const float dz = fabsf(d.z) < e ? __builtin_copysignf(e, d.z) : d.z;
  const F3 ni = f3(rcp(dx), rcp(dy), rcp(dz));
  const F3 oi = f3(o.x * ni.x, o.y * ni.y, o.z * ni.z);
  const int lane = (int)__lane_id();
  int stack = 0;
  int sp = 0;
  int node = root;
  for (int iter = 0; iter < p.max_iters; ++iter) {
    RT_STAMP(t_node);
    const Bvh4Node nd = cp(p.nodes4)[node];
    if constexpr (COUNT) {
      ws.v[STAT_NODE_FETCH] += 1u;
      ws.v[STAT_LANE_NODES] += pc(bal(active));
    }
    float tn[4];
    bool h[4];
    unsigned long long m[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float ax = __builtin_fmaf(nd.lo[0][k], ni.x, -oi.x), bx = __builtin_fmaf(nd.hi[0][k], ni.x, -oi.x);
      const float ay = __builtin_fmaf(nd.lo[1][k], ni.y, -oi.y), by = __builtin_fmaf(nd.hi[1][k], ni.y, -oi.y);
      const float az = __builtin_fmaf(nd.lo[2][k], ni.z, -oi.z), bz = __builtin_fmaf(nd.hi[2][k], ni.z, -oi.z);
      tn[k] = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), 0.0f));
      const float tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fminf(fmaxf(az, bz), tbest));
      h[k] = active && tn[k] <= tf * 1.0000004f;
      m[k] = nd.count[k] >= 0 ? bal(h[k]) : 0ull;
    }
#ifdef RTMI_STAMPS
    { RT_STAMP(t_slab); RT_ACC(8, t_node, t_slab); }
#endif
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (nd.count[k] > 0 && m[k]) {
        RT_STAMP(t_leaf);
        if constexpr (COUNT) {
          ws.v[STAT_TRI_FETCH] += (unsigned int)nd.count[k];
          ws.v[STAT_LANE_TRIS] += pc(m[k]) * (unsigned int)nd.count[k];
        }
        leaf(p, nd.child[k], nd.count[k], h[k], o, d, tbest, best_id);
        if (anyhit) active = active && best_id < 0;
        m[k] = 0ull;
#ifdef RTMI_STAMPS
        { RT_STAMP(t_leaf_end); RT_ACC(6, t_leaf, t_leaf_end); }
#endif
      }
    }
    if (anyhit && bal(active) == 0ull) break;
    // order the internal children hit by any lane
    const unsigned long long live = bal(active);
    const int lead = live ? (int)__builtin_ctzll(live) : 0;
    unsigned key[4];
    int cn[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned tk = (unsigned)__builtin_amdgcn_readlane(__float_as_int(tn[k]), lead);
      key[k] = m[k] ? (((m[k] >> lead) & 1ull) ? tk : 0x7f000000u) : 0xffffffffu;
      cn[k] = nd.child[k];
    }
    cswap(key[0], cn[0], key[1], cn[1]);
    cswap(key[2], cn[2], key[3], cn[3]);
    cswap(key[0], cn[0], key[2], cn[2]);
    cswap(key[1], cn[1], key[3], cn[3]);
    cswap(key[1], cn[1], key[2], cn[2]);
    if (key[0] == 0xffffffffu) {
      if (sp == 0) break;
      --sp;
      node = __builtin_amdgcn_readlane(stack, sp);
    } else {
      node = cn[0];
#pragma unroll
      for (int k = 3; k >= 1; --k) {
        if (key[k] != 0xffffffffu) {
          stack = (lane == sp) ? cn[k] : stack;
          ++sp;
        }
      }
    }
  }
#ifdef RTMI_STAMPS
  { RT_STAMP(t_exit); RT_ACC(5, t_enter, t_exit); }
#endif
}

// trace (renderer.nim:47-67): linear closest hit over the objects in order.
template <bool COUNT>
__device__ __forceinline__ Hit trace(const FastParams& p, F3 o, F3 d, float tmax, bool active, bool anyhit,
                                     Stats32& ws) {
  Hit h{-1, -1, tmax};
  ws.v[STAT_TESTS] += pc(bal(active)) * (unsigned int)p.nobj;
  for (int i = 0; i < p.nobj; ++i) {
    const FObj ob = cp(p.objs)[i];
    F3 ro, rd;
    to_object(p, ob, i, o, d, ro, rd);
    float t;
    int tri = -1;
    if (ob.type == GEOM_PLANE) {
      t = plane(ro, rd);
    } else if (ob.type == GEOM_SPHERE) {
      t = sphere(ob.r, ro, rd);
    } else if (ob.type == GEOM_BOX) {
      t = aabb(ob.lo, ob.hi, ro, f3(rcp(rd.x), rcp(rd.y), rcp(rd.z)));
    } else {
      const FMesh m = cp(p.meshes)[ob.mesh];
      // TriangleMesh.intersect (geom.nim:339-358): a ray starting inside
      // the mesh AABB misses; otherwise the closest face.
      const float gate = aabb(m.lo, m.hi, ro, f3(rcp(rd.x), rcp(rd.y), rcp(rd.z)));
      const bool in = gate >= 0.0f;
      float tb = h.t;
      int best = -1;
#if RTMI_BVH4
      if (m.root >= 0) traverse4<COUNT>(p, m.root, ro, rd, active && in, anyhit, tb, best, ws);
#else
      if (m.root2 >= 0) traverse2<COUNT>(p, m.root2, ro, rd, active && in, anyhit, tb, best, ws);
#endif
      t = !in ? -finf() : (best >= 0 ? tb : finf());
      tri = best;
    }
    const bool upd = active && t >= 0.0f && t < h.t;
    ws.v[STAT_HITS] += pc(bal(upd));
    if (upd) {
      h.t = t;
      h.obj = i;
      h.tri = tri;
    }
  }
  return h;
}

// normal(*) (geom.nim:361-379) for analytic geometry, object space.
__device__ __forceinline__ F3 analytic_normal(const FObj& ob, F3 ho) {
  if (ob.type == GEOM_SPHERE) {
    const float r = rsq(dot3(ho, ho));
    return f3(ho.x * r, ho.y * r, ho.z * r);
  }
  if (ob.type == GEOM_BOX) {
    const float cx = (ob.lo[0] + ob.hi[0]) * 0.5f, cy = (ob.lo[1] + ob.hi[1]) * 0.5f,
                cz = (ob.lo[2] + ob.hi[2]) * 0.5f;
    const float qx = (ho.x - cx) * rcp(fabsf((ob.lo[0] - ob.hi[0]) * 0.5f));
    const float qy = (ho.y - cy) * rcp(fabsf((ob.lo[1] - ob.hi[1]) * 0.5f));
    const float qz = (ho.z - cz) * rcp(fabsf((ob.lo[2] - ob.hi[2]) * 0.5f));
    // 1.0001 instead of 1.000001: a float32 hit point is good to ~1e-5 of
    // the box size; fall back to the dominant axis rather than a NaN normal.
    F3 n = f3(truncf(qx * 1.0001f), truncf(qy * 1.0001f), truncf(qz * 1.0001f));
    if (n.x == 0.0f && n.y == 0.0f && n.z == 0.0f) {
      const float ax = fabsf(qx), ay = fabsf(qy), az = fabsf(qz);
      if (ax >= ay && ax >= az) n.x = qx < 0.0f ? -1.0f : 1.0f;
      else if (ay >= az) n.y = qy < 0.0f ? -1.0f : 1.0f;
      else n.z = qz < 0.0f ? -1.0f : 1.0f;
    }
    const float r = rsq(dot3(n, n));
    return f3(n.x * r, n.y * r, n.z * r);
  }
  return f3(0.0f, 1.0f, 0.0f);  // plane
}

// One camera sample: trace + shade (renderer.nim:71-127), reflections as a
// loop of levels with forward weights.
template <bool COUNT>
__device__ __forceinline__ F3 shade_path(const FastParams& p, F3 o, F3 d, bool active, Stats32& ws) {
  const bool anyhit_shadows = (p.flags & RT_DEV_FLAG_ANYHIT) != 0;
  bool act = active;
  int depth = 1;
  F3 acc = f3(0.0f, 0.0f, 0.0f);
  float w = 1.0f;
  for (int lev = 0; lev < kMaxShadeLevels; ++lev) {
    if (bal(act) == 0ull) break;
    const Hit hit = trace<COUNT>(p, o, d, finf(), act, false, ws);
#ifdef RTMI_EXP_PRIMARY_ONLY
    return f3(hit.t, (float)hit.obj, (float)hit.tri);
#endif
    if (act && hit.obj < 0) acc = f3(acc.x + w * p.bg[0], acc.y + w * p.bg[1], acc.z + w * p.bg[2]);
    const bool lit = act && hit.obj >= 0;
    const F3 hw = f3(__builtin_fmaf(d.x, hit.t, o.x), __builtin_fmaf(d.y, hit.t, o.y), __builtin_fmaf(d.z, hit.t, o.z));
    F3 N = f3(0.0f, 0.0f, 0.0f);
    F3 alb = f3(0.0f, 0.0f, 0.0f);
    float refl = 0.0f;
    unsigned long long pending = bal(lit);
    while (pending) {  // one pass per distinct object hit by the wave
      const int lead = (int)__builtin_ctzll(pending);
      const int oi = __builtin_amdgcn_readlane(hit.obj, lead);
      const bool mine = lit && hit.obj == oi;
      pending &= ~bal(mine);
      const FObj ob = cp(p.objs)[oi];
      const RT_CONST FObjX& ox = cp(p.objx)[oi];
      if (mine) {
        F3 n;
        if (ob.type == GEOM_MESH) {
          const float* fn = p.normals + 3 * (size_t)(ox.normal_base + hit.tri);
          n = f3(fn[0], fn[1], fn[2]);
        } else {
          F3 ho, unused;
          to_object(p, ob, oi, hw, f3(0.0f, 0.0f, 0.0f), ho, unused);
          n = analytic_normal(ob, ho);
        }
        if (ob.xf == XF_GENERAL) {  // object_to_world * n, not re-normalised
          const float* m = ox.o2w;
          N = f3(__builtin_fmaf(m[0], n.x, __builtin_fmaf(m[3], n.y, m[6] * n.z)),
                 __builtin_fmaf(m[1], n.x, __builtin_fmaf(m[4], n.y, m[7] * n.z)),
                 __builtin_fmaf(m[2], n.x, __builtin_fmaf(m[5], n.y, m[8] * n.z)));
        } else {
          N = n;
        }
        alb = f3(ox.albedo_pi[0], ox.albedo_pi[1], ox.albedo_pi[2]);
        refl = ox.refl;
      }
    }
    F3 local = f3(0.0f, 0.0f, 0.0f);
    const F3 so = f3(__builtin_fmaf(N.x, p.bias, hw.x), __builtin_fmaf(N.y, p.bias, hw.y),
                     __builtin_fmaf(N.z, p.bias, hw.z));
    for (int li = 0; li < p.nlight; ++li) {
      const FLight L = cp(p.lights)[li];
      F3 sd, I;
      float dist;
      if (L.type == LIGHT_POINT) {  // light.nim:52-62
        const F3 lv = f3(hw.x - L.v[0], hw.y - L.v[1], hw.z - L.v[2]);
        const float r2 = dot3(lv, lv);
        const float rr = rsq(r2);
        sd = f3(-lv.x * rr, -lv.y * rr, -lv.z * rr);
        const float k = rcp(12.566370614359172f * r2);
        I = f3(L.ci[0] * k, L.ci[1] * k, L.ci[2] * k);
        dist = r2 * rr;
      } else {  // light.nim:46-50
        sd = f3(-L.v[0], -L.v[1], -L.v[2]);
        I = f3(L.ci[0], L.ci[1], L.ci[2]);
        dist = finf();
      }
      ws.v[STAT_SHADOW] += pc(bal(lit));
      const Hit sh = trace<COUNT>(p, so, sd, dist, lit, anyhit_shadows, ws);
      if (lit && sh.obj < 0) {  // shadeDiffuse (shader.nim:12-17)
        const float ndl = fmaxf(dot3(N, sd), 0.0f);
        local = f3(__builtin_fmaf(alb.x * I.x, ndl, local.x), __builtin_fmaf(alb.y * I.y, ndl, local.y),
                   __builtin_fmaf(alb.z * I.z, ndl, local.z));
      }
    }
    const bool reflect = lit && refl > 0.0f && depth <= p.max_depth;
    const float wl = reflect ? w * (1.0f - refl) : w;
    if (lit) acc = f3(__builtin_fmaf(wl, local.x, acc.x), __builtin_fmaf(wl, local.y, acc.y),
                      __builtin_fmaf(wl, local.z, acc.z));
    ws.v[STAT_REFL] += pc(bal(reflect));
    if (reflect) {  // renderer.nim:109-118
      w = w * refl;
      const float ndi = 2.0f * dot3(N, d);
      const F3 rd = f3(d.x - N.x * ndi, d.y - N.y * ndi, d.z - N.z * ndi);
      o = f3(__builtin_fmaf(rd.x, p.bias, hw.x), __builtin_fmaf(rd.y, p.bias, hw.y), __builtin_fmaf(rd.z, p.bias, hw.z));
      d = rd;
      ++depth;
    }
    act = reflect;
  }
  return acc;
}

__device__ __forceinline__ void flush(Stats32& ws, unsigned long long& tot, int lane) {
#pragma unroll
  for (int k = 0; k < kStatSlots; ++k) {
    tot += (lane == k) ? (unsigned long long)ws.v[k] : 0ull;
    ws.v[k] = 0u;
  }
}

template <bool COUNT>
__global__ __launch_bounds__(256) void k_render_fast(const FastParams p) {
  const int lane = (int)__lane_id();
  const int wave = (int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const int nwaves = (int)(gridDim.x * (blockDim.x >> 6));
  const int L = p.lanes_per_px;
  const int sub = lane & (L - 1);
  const int pix = lane >> p.log2_lanes;
  const int tpx = pix % p.tile_x, tpy = pix / p.tile_x;
  const int iters = (p.spp + L - 1) / L;
  const bool grid_aa = p.aa_kind != 0;
  const int m = p.grid_m;
  const int si0 = sub % m, sj0 = sub / m;  // grid coordinates of this lane's first sample
  const int dli = L % m, dlj = L / m;      // advance of the grid coordinates per iteration
  Stats32 ws;
#pragma unroll
  for (int k = 0; k < kStatSlots; ++k) ws.v[k] = 0u;
  unsigned long long tot = 0ull;

  for (int g = wave; g < p.ngroups; g += nwaves) {
    const int gx = g % p.tiles_x, gy = g / p.tiles_x;
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
    F3 acc = f3(0.0f, 0.0f, 0.0f);
    int bi = 0, bj = 0;  // grid coordinates of sample it*L (wave-uniform)
    for (int it = 0; it < iters; ++it) {
      const bool sv = valid && it * L + sub < p.spp;
      float px = (float)x, py = (float)y;
      if (grid_aa) {  // grid() sampling.nim:5-18
        int si = bi + si0, sj = bj + sj0;
        if (si >= m) {
          si -= m;
          sj += 1;
        }
        px += __builtin_fmaf((float)si, p.sample_step, p.sample_off);
        py += __builtin_fmaf((float)sj, p.sample_step, p.sample_off);
      }
      // castPrimaryRay (renderer.nim:31-44), constants folded on the host
      // ((2 x r)/w - r) f == (x - w/2) (2 r f / w): exact 0 on the centre
      // column / row, as the reference's own formula gives there
      const float cx = (px - p.cam_b) * p.cam_a;
      const float cy = (p.cam_d - py) * p.cam_c;
      const float rl = rsq(__builtin_fmaf(cx, cx, __builtin_fmaf(cy, cy, 1.0f)));
      const F3 d = f3((cx * p.cam[3] + cy * p.cam[6] - p.cam[9]) * rl, (cx * p.cam[4] + cy * p.cam[7] - p.cam[10]) * rl,
                      (cx * p.cam[5] + cy * p.cam[8] - p.cam[11]) * rl);
      const F3 o = f3(p.cam[0], p.cam[1], p.cam[2]);
      ws.v[STAT_PRIMARY] += pc(bal(sv));
      RT_STAMP(t_s0);
      const F3 c = shade_path<COUNT>(p, o, d, sv, ws);
#ifdef RTMI_STAMPS
      { RT_STAMP(t_s1); RT_ACC(7, t_s0, t_s1); }
#endif
      if (sv) acc = grid_aa ? f3(acc.x + c.x, acc.y + c.y, acc.z + c.z) : c;
      bi += dli;
      bj += dlj;
      if (bi >= m) {
        bi -= m;
        bj += 1;
      }
    }
    flush(ws, tot, lane);
    for (int off = 1; off < L; off <<= 1) {
      acc.x += __shfl_xor(acc.x, off);
      acc.y += __shfl_xor(acc.y, off);
      acc.z += __shfl_xor(acc.z, off);
    }
    if (valid && sub == 0) {
      if (grid_aa) acc = f3(acc.x * p.inv_len, acc.y * p.inv_len, acc.z * p.inv_len);
      if (p.mode == 0 && p.step > 1) {
        const int xe = min(x + p.step, p.width), ye = min(y + p.step, p.height);
        for (int yy = y; yy < ye; ++yy)
          for (int xx = x; xx < xe; ++xx) {
            float* q = p.fb + ((size_t)yy * p.width + xx) * 3;
            q[0] = acc.x; q[1] = acc.y; q[2] = acc.z;
          }
      } else {
        float* q = p.fb + ((size_t)out_row * p.width + x) * 3;
        q[0] = acc.x; q[1] = acc.y; q[2] = acc.z;
      }
    }
  }
  if (lane < kStatSlots) p.partials[(size_t)wave * kStatSlots + lane] = tot;
}

}  // namespace fast
}  // namespace rtmi
