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
#include "rt_sampling.h"

#ifndef RT_CONST
#if defined(__HIP_DEVICE_COMPILE__)
#define RT_CONST __attribute__((address_space(4)))  // scalar (constant) loads
#else
#define RT_CONST
#endif
#endif



#include "rt_occupancy.h"

namespace rtmi {
namespace fast {

// Scene-feature mask of a kernel instantiation: code for a feature whose bit
// is clear is removed at compile time (the host picks the smallest
// instantiation covering the scene, rtmi.cpp feature_mask()).
enum : unsigned {
  F_SPHERE = 1u, F_BOX = 2u, F_PLANE = 4u, F_MESH = 8u,
  F_XF_GENERAL = 16u,  // rotations / scales (identity and translation always)
  F_POINT = 32u,       // point lights
  F_REFLECT = 64u,     // reflective materials
  F_STOCHASTIC = 128u, // jittered / (correlated) multi-jittered sampling
  F_ALL = 255u
};

template <class T>
__device__ __forceinline__ const RT_CONST T* cp(const T* p) {
  return (const RT_CONST T*)(p);
}

// Record i of a small scene array (objects, lights: < 2^25 records) at a
// 32-bit byte offset: s_load with an SGPR offset, one shift instead of the
// 64-bit address arithmetic per object / light visit.
template <class T>
__device__ __forceinline__ const RT_CONST T& at(const T* base, int i) {
  return *(const RT_CONST T*)((const RT_CONST char*)base + (unsigned)i * (unsigned)sizeof(T));
}

// Work items of a two-class launch's list: its entry count as this call's
// k_frame_records counted it on the device (n, rt_frame.h; per_item entries
// per item), or the host's item count when the list is not counted.
__device__ __forceinline__ int list_items(const int32_t* n, int host_items, int per_item) {
  return n ? (cp(n)[0] + per_item - 1) / per_item : host_items;
}

__device__ __forceinline__ unsigned long long bal(bool p) { return __builtin_amdgcn_ballot_w64(p); }
// Lane masks straight from a v_cmp (llvm.amdgcn.fcmp: ordered >= / <) and a
// mask back to a per-lane predicate (llvm.amdgcn.inverse.ballot): a ballot of
// a compound bool otherwise materialises it in a VGPR (v_cndmask 0/1 +
// v_cmp_ne) before the popcount.
#ifndef RTMI_FCMP_MASKS
#define RTMI_FCMP_MASKS 1
#endif
__device__ __forceinline__ unsigned long long m_ge(float a, float b) { return __builtin_amdgcn_fcmpf(a, b, 3); }
__device__ __forceinline__ unsigned long long m_lt(float a, float b) { return __builtin_amdgcn_fcmpf(a, b, 4); }
__device__ __forceinline__ bool lane_in(unsigned long long m) { return __builtin_amdgcn_inverse_ballot_w64(m); }
__device__ __forceinline__ unsigned int pc(unsigned long long m) { return (unsigned int)__builtin_popcountll(m); }
__device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float rsq(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float finf() { return __builtin_huge_valf(); }

// Kernel parameters are read through this pointer into the kernarg segment,
// re-laundered (opaque to the optimizer) once per pixel group, sample and
// light: each field is then re-read with a scalar load near its use instead
// of being hoisted to the kernel entry and pinned in SGPRs for the whole
// kernel (which spilled ~100 SGPRs into VGPR lanes and cost a v_readlane per
// use). Inside traverse() the pointer is invariant, so the node / triangle
// base addresses stay hoisted off the fetch chain.
using KP = const RT_CONST FastParams*;
__device__ __forceinline__ KP params() {
  KP q = (KP)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(q));
  return q;
}

struct F3 {
  float x, y, z;
};

template <bool B>
struct Bool {
  static constexpr bool value = B;
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
template <unsigned F>
__device__ __forceinline__ void to_object(KP p, const FObj& ob, int i, F3 o, F3 d, F3& ro,
                                          F3& rd) {
  // identity and translation alike: the identity's translation is 0 (three
  // adds instead of a scalar compare + selects per object visit)
  if (!(F & F_XF_GENERAL) || ob.xf != XF_GENERAL) {
    ro = f3(o.x + ob.t[0], o.y + ob.t[1], o.z + ob.t[2]);
    rd = d;
  } else {
    const RT_CONST FObjX& x = at(p->objx, i);
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

// A TriFast record as ONE s_load_dwordx16 (the compiler otherwise splits the
// record into per-field loads — up to eight SMEM instructions per face in
// the batched list searches — since a face test reads 13 of its 16 dwords):
// the pad dwords are marked live so the load stays whole.
struct TriRegs {
  float v0[3], e2[3], e1n[3], nn[3];
  unsigned int id;
};
__device__ __forceinline__ TriRegs load_tri(const RT_CONST TriFast* t) {
  using V16 = unsigned int __attribute__((ext_vector_type(16)));
  const V16 r = *(const RT_CONST V16*)t;
  asm volatile("" ::"s"(r[7]), "s"(r[11]), "s"(r[15]));
  TriRegs T;
  T.v0[0] = __uint_as_float(r[0]), T.v0[1] = __uint_as_float(r[1]), T.v0[2] = __uint_as_float(r[2]);
  T.id = r[3];
  T.e2[0] = __uint_as_float(r[4]), T.e2[1] = __uint_as_float(r[5]), T.e2[2] = __uint_as_float(r[6]);
  T.e1n[0] = __uint_as_float(r[8]), T.e1n[1] = __uint_as_float(r[9]), T.e1n[2] = __uint_as_float(r[10]);
  T.nn[0] = __uint_as_float(r[12]), T.nn[1] = __uint_as_float(r[13]), T.nn[2] = __uint_as_float(r[14]);
  return T;
}

// Closest hit as ONE 64-bit key: float bits of t in the high word, the
// triangle's face index in the low word. For t >= 0 the float bits order like
// unsigned integers, so key order is the reference's "smaller t, then lower
// face index" order (geom.nim:339-358 keeps the first, i.e. lowest-index,
// face on a tie); a negative or NaN t sorts above +inf and is never accepted.
// One v_cmp_lt_u64 + three v_cndmask replace the compare/tie-break mask
// algebra (which cost SALU s_and/s_or per triangle).
__device__ __forceinline__ unsigned long long tkey(float t, unsigned int lo) {
  return ((unsigned long long)__float_as_uint(t) << 32) | lo;
}

// rayTriangleIntersectFast (geom.nim:283-336), single-sided, on the TriFast
// record (rt_common.h): with c = (o - v0) x d and nn = -(e1 x e2),
//   det = d.nn, u*det = e2.c, v*det = (-e1).c, t = (o - v0).nn / (-det)
// (scalar triple-product identities of the reference's p = d x e2,
// q = tvec x e1 form). The barycentric range is tested unscaled in one min:
// u >= 0, v >= 0, u + v <= 1 (u <= 1 is implied), det >= 1e-6.
template <class TR>
__device__ __forceinline__ void tri_test(const TR& T, F3 o, F3 d, unsigned long long& key, float& tc) {
  const float tx = o.x - T.v0[0], ty = o.y - T.v0[1], tz = o.z - T.v0[2];
  const float cx = __builtin_fmaf(ty, d.z, -tz * d.y);
  const float cy = __builtin_fmaf(tz, d.x, -tx * d.z);
  const float cz = __builtin_fmaf(tx, d.y, -ty * d.x);
  const float u = __builtin_fmaf(T.e2[0], cx, __builtin_fmaf(T.e2[1], cy, T.e2[2] * cz));
  const float v = __builtin_fmaf(T.e1n[0], cx, __builtin_fmaf(T.e1n[1], cy, T.e1n[2] * cz));
  const float det = __builtin_fmaf(T.nn[0], d.x, __builtin_fmaf(T.nn[1], d.y, T.nn[2] * d.z));
  const float tt = __builtin_fmaf(T.nn[0], tx, __builtin_fmaf(T.nn[1], ty, T.nn[2] * tz));
  const float t = tt * rcp(-det);
  const float g = fminf(fminf(fminf(u, v), det - (u + v)), det - 0.000001f);
  const float ts = g >= 0.0f ? t : -1.0f;
  const unsigned long long k = tkey(ts, (unsigned int)T.id);
  const bool acc = k < key;
  key = acc ? k : key;
  tc = acc ? ts : tc;
}

// Shadow-ray tests on a face's LTri record for the ray's distant light
// (rt_common.h): u, v, t are affine in the ray origin, so a test is 9 FMAs
// and the barycentric range in one min (u >= 0, v >= 0, u + v <= 1; the
// det >= 1e-6 cull is folded into the record). Every float32 path tests a
// shadow ray to a light with records this way (list searches, BVH leaves,
// batched and one-sample loops), so they all form the same t bit for bit.
struct LRegs {
  float p[3], cu, q[3], cv, tv[3], ct;
  unsigned int id;
};
__device__ __forceinline__ LRegs load_ltri(const RT_CONST LTri* t) {
  using V16 = unsigned int __attribute__((ext_vector_type(16)));
  const V16 r = *(const RT_CONST V16*)t;
  asm volatile("" ::"s"(r[13]), "s"(r[14]), "s"(r[15]));
  LRegs L;
  L.p[0] = __uint_as_float(r[0]), L.p[1] = __uint_as_float(r[1]), L.p[2] = __uint_as_float(r[2]);
  L.cu = __uint_as_float(r[3]);
  L.q[0] = __uint_as_float(r[4]), L.q[1] = __uint_as_float(r[5]), L.q[2] = __uint_as_float(r[6]);
  L.cv = __uint_as_float(r[7]);
  L.tv[0] = __uint_as_float(r[8]), L.tv[1] = __uint_as_float(r[9]), L.tv[2] = __uint_as_float(r[10]);
  L.ct = __uint_as_float(r[11]);
  L.id = r[12];
  return L;
}
// t of the hit, or -1 (no hit: outside the face, or det culled)
template <class LR>
__device__ __forceinline__ float ltri_t(const LR& L, F3 o) {
  const float u = __builtin_fmaf(L.p[0], o.x, __builtin_fmaf(L.p[1], o.y, __builtin_fmaf(L.p[2], o.z, L.cu)));
  const float v = __builtin_fmaf(L.q[0], o.x, __builtin_fmaf(L.q[1], o.y, __builtin_fmaf(L.q[2], o.z, L.cv)));
  const float t = __builtin_fmaf(L.tv[0], o.x, __builtin_fmaf(L.tv[1], o.y, __builtin_fmaf(L.tv[2], o.z, L.ct)));
  const float g = fminf(fminf(u, v), 1.0f - (u + v));
  return g >= 0.0f ? t : -1.0f;
}
template <class LR>
__device__ __forceinline__ void ltri_test(const LR& L, F3 o, unsigned long long& key, float& tc) {
  const float ts = ltri_t(L, o);
  const unsigned long long k = tkey(ts, (unsigned int)L.id);
  const bool acc = k < key;
  key = acc ? k : key;
  tc = acc ? ts : tc;
}
// the records of shadow rays to distant light `light` (byte offsets are the
// faces' TriFast offsets), or nullptr when the light has none
__device__ __forceinline__ const char* lrec_of(KP p, int light) {
  if (light < 0 || light >= 32 || !((p->lrec_mask >> light) & 1u)) return nullptr;
  return (const char*)(p->lrec_base + (uint64_t)light * (uint64_t)p->lrec_stride);
}

#ifndef RTMI_GRID_REC
#define RTMI_GRID_REC 1
#endif
// The cell-ordered records of a light's grid, aligned with its entries
// (p->grid_ent + G.ent_base): list_search_batch's lb under RTMI_GRID_REC.
__device__ __forceinline__ const char* grid_rec_of(KP p, int light, const LightGrid& G) {
  return RTMI_GRID_REC ? (const char*)(p->grid_rec + G.ent_base) : lrec_of(p, light);
}

// A record of the float32 tree (FastParams.tree) at a byte offset: one scalar
// base + a 32-bit SGPR offset (s_load ... soffset), no 64-bit address
// arithmetic on the traversal's dependent chain.
template <class T>
__device__ __forceinline__ const RT_CONST T* rec(KP p, int off) {
  return (const RT_CONST T*)((const RT_CONST char*)p->tree + (unsigned)off);
}

// Leaf: the n (1..kLeafMax, wave-uniform) triangles starting at byte offset
// `first` of the tree.
__device__ __forceinline__ void leaf(KP p, int first, int n, F3 o, F3 d, unsigned long long& key,
                                     float& tc, const char* lb = nullptr) {
  if (lb) {  // a shadow ray to a light with LTri records
    const RT_CONST LTri* l = (const RT_CONST LTri*)(lb + (unsigned)first);
    ltri_test(load_ltri(l), o, key, tc);
#pragma unroll
    for (int k = 1; k < kLeafMax; ++k) {
      if (k >= n) break;
      ltri_test(load_ltri(l + k), o, key, tc);
    }
    return;
  }
  const RT_CONST TriFast* t = rec<TriFast>(p, first);
  tri_test(load_tri(t), o, d, key, tc);
#pragma unroll
  for (int k = 1; k < kLeafMax; ++k) {
    if (k >= n) break;
    tri_test(load_tri(t + k), o, d, key, tc);
  }
}

// Wave-coherent closest hit over one mesh BVH2 (64-B nodes, both child boxes
// per scalar fetch). Per lane: `tc` is the box-culling limit (the current
// best t; -1 for lanes that take no part, so `active` never enters a lane
// mask) and `key` the best (t, face) so far. Lanes step through the same node
// sequence: a child is visited when any lane's ray hits its box; both hit ->
// the nearer (majority vote) first, the other onto a 64-entry stack held one
// entry per lane in a single VGPR. Every child reference is valid (the
// builder never emits an empty child), and no iteration guard is needed: a
// traversal visits each node at most once.
// early/stop: exact early exit for shadow rays (trace()): a lane
// retires once its best t <= stop.
// Box-test form of a ray: ni = 1/d with components below 1e-20 in magnitude
// replaced by +-1e-20 (finite slabs, no 0 * inf), oi = o * ni; a slab plane
// x = c is crossed at fma(c, ni.x, -oi.x).
struct SlabRay {
  F3 ni, oi;
};
__device__ __forceinline__ SlabRay slab_ray(F3 o, F3 d) {
  const float e = 1e-20f;
  const float dx = fabsf(d.x) < e ? __builtin_copysignf(e, d.x) : d.x;
  const float dy = fabsf(d.y) < e ? __builtin_copysignf(e, d.y) : d.y;
  const float dz = fabsf(d.z) < e ? __builtin_copysignf(e, d.z) : d.z;
  SlabRay r;
  r.ni = f3(rcp(dx), rcp(dy), rcp(dz));
  r.oi = f3(o.x * r.ni.x, o.y * r.ni.y, o.z * r.ni.z);
  return r;
}

// The search state (key, tc) is the caller's (trace()): lanes with tc < 0
// take no part (never entered, retired, or done by a bin search).
template <bool COUNT>
__device__ __forceinline__ void traverse(KP p, int root, F3 o, F3 d, SlabRay sr, bool early, float stop,
                                         unsigned long long& key, float& tc, Stats32& ws,
                                         const char* lb = nullptr) {
  if (bal(tc >= 0.0f) == 0ull) return;
  RT_STAMP(t_enter);
  const F3 ni = sr.ni, oi = sr.oi;
  const int lane = (int)__lane_id();
  int stack = 0;
  int sp = 0;
  int node = root;
  // COUNT only: the lanes whose own ray hit the current node's box at its
  // parent (per-ray visits); far children's masks are
  // stacked alongside (two more VGPR stacks, diagnostic kernel only)
  unsigned long long vm = 0ull;
  int mlo = 0, mhi = 0;
  if constexpr (COUNT) vm = bal(tc >= 0.0f);
  for (;;) {
    const BvhNode nd = *rec<BvhNode>(p, node);
    if constexpr (COUNT) {
      ws.v[STAT_NODE_FETCH] += 1u;
      ws.v[STAT_LANE_NODES] += pc(vm);
    }
    const float ax0 = __builtin_fmaf(nd.lo0[0], ni.x, -oi.x), bx0 = __builtin_fmaf(nd.hi0[0], ni.x, -oi.x);
    const float ay0 = __builtin_fmaf(nd.lo0[1], ni.y, -oi.y), by0 = __builtin_fmaf(nd.hi0[1], ni.y, -oi.y);
    const float az0 = __builtin_fmaf(nd.lo0[2], ni.z, -oi.z), bz0 = __builtin_fmaf(nd.hi0[2], ni.z, -oi.z);
    const float ax1 = __builtin_fmaf(nd.lo1[0], ni.x, -oi.x), bx1 = __builtin_fmaf(nd.hi1[0], ni.x, -oi.x);
    const float ay1 = __builtin_fmaf(nd.lo1[1], ni.y, -oi.y), by1 = __builtin_fmaf(nd.hi1[1], ni.y, -oi.y);
    const float az1 = __builtin_fmaf(nd.lo1[2], ni.z, -oi.z), bz1 = __builtin_fmaf(nd.hi1[2], ni.z, -oi.z);
    const float tn0 = fmaxf(fmaxf(fminf(ax0, bx0), fminf(ay0, by0)), fmaxf(fminf(az0, bz0), 0.0f));
    const float tf0 = fminf(fminf(fmaxf(ax0, bx0), fmaxf(ay0, by0)), fminf(fmaxf(az0, bz0), tc));
    const float tn1 = fmaxf(fmaxf(fminf(ax1, bx1), fminf(ay1, by1)), fmaxf(fminf(az1, bz1), 0.0f));
    const float tf1 = fminf(fminf(fmaxf(ax1, bx1), fmaxf(ay1, by1)), fminf(fmaxf(az1, bz1), tc));
    unsigned long long m0 = bal(tn0 <= tf0 * 1.0000004f);
    unsigned long long m1 = bal(tn1 <= tf1 * 1.0000004f);
    if (nd.n0 > 0) {
      if (m0) {
        if constexpr (COUNT) {
          ws.v[STAT_TRI_FETCH] += (unsigned int)nd.n0;
          ws.v[STAT_LANE_TRIS] += pc(m0) * (unsigned int)nd.n0;
        }
        leaf(p, nd.c0, nd.n0, o, d, key, tc, lb);
        if (early) tc = tc <= stop ? -1.0f : tc;
      }
      m0 = 0ull;
    }
    if (nd.n1 > 0) {
      if (m1) {
        if constexpr (COUNT) {
          ws.v[STAT_TRI_FETCH] += (unsigned int)nd.n1;
          ws.v[STAT_LANE_TRIS] += pc(m1) * (unsigned int)nd.n1;
        }
        leaf(p, nd.c1, nd.n1, o, d, key, tc, lb);
        if (early) tc = tc <= stop ? -1.0f : tc;
      }
      m1 = 0ull;
    }
    if (m0 && m1) {
      const unsigned long long both = m0 & m1;
      const bool first0 = pc(bal(tn0 <= tn1) & both) * 2u >= pc(both);
      const int near = first0 ? nd.c0 : nd.c1;
      const int far = first0 ? nd.c1 : nd.c0;
      stack = (lane == sp) ? far : stack;
      if constexpr (COUNT) {
        const unsigned long long fm = first0 ? m1 : m0;
        mlo = (lane == sp) ? (int)(unsigned int)fm : mlo;
        mhi = (lane == sp) ? (int)(unsigned int)(fm >> 32) : mhi;
        vm = first0 ? m0 : m1;
      }
      ++sp;
      node = near;
    } else if (m0) {
      node = nd.c0;
      if constexpr (COUNT) vm = m0;
    } else if (m1) {
      node = nd.c1;
      if constexpr (COUNT) vm = m1;
    } else {
      if (sp == 0) break;
      if (early && bal(tc >= 0.0f) == 0ull) break;
      --sp;
      node = __builtin_amdgcn_readlane(stack, sp);
      if constexpr (COUNT)
        vm = (unsigned long long)(unsigned int)__builtin_amdgcn_readlane(mlo, sp) |
             ((unsigned long long)(unsigned int)__builtin_amdgcn_readlane(mhi, sp) << 32);
    }
  }
#ifdef RTMI_STAMPS
  { RT_STAMP(t_exit); RT_ACC(5, t_enter, t_exit); }
#endif
}

// The faces listed at ent[b, e) (a pixel list or a light-grid cell, rt_bins.h)
// against every lane's ray, with the traversal's key / early-exit rules.
// ent is padded, so the four-record read-ahead stays inside the array.
template <bool COUNT>
__device__ __forceinline__ void list_search(KP p, const int32_t* ent, int b, int e, F3 o, F3 d, bool early,
                                            float stop, unsigned long long& key, float& tc, Stats32& ws,
                                            const char* lb = nullptr) {
  if constexpr (COUNT) {
    ws.v[STAT_TRI_FETCH] += (unsigned int)(e - b);
    ws.v[STAT_LANE_TRIS] += pc(bal(tc >= 0.0f)) * (unsigned int)(e - b);
  }
#ifdef RTMI_DIAG_NOLIST
  return;  // diagnostic build only: the binned searches' share of the frame
#endif
  auto test = [&](int off) {
    if (lb) ltri_test(load_ltri((const RT_CONST LTri*)(lb + (unsigned)off)), o, key, tc);
    else tri_test(load_tri(rec<TriFast>(p, off)), o, d, key, tc);
  };
  if (early && b < e) {  // a light cell's first face alone (the one covering most of the cell)
    test(cp(ent)[b]);
    tc = tc <= stop ? -1.0f : tc;
    if (bal(tc >= 0.0f) == 0ull) return;
    ++b;
  }
  for (int k = b; k < e; k += 4) {
    const RT_CONST int32_t* q = cp(ent) + k;
    const int r0 = q[0], r1 = q[1], r2 = q[2], r3 = q[3];
    test(r0);
    if (k + 1 < e) test(r1);
    if (k + 2 < e) test(r2);
    if (k + 3 < e) test(r3);
    if (early) {
      tc = tc <= stop ? -1.0f : tc;
      if (bal(tc >= 0.0f) == 0ull) break;
    }
  }
}

// t of analytic object i in world space, -inf on a miss (Sphere / Plane /
// Box .intersect, geom.nim:215-248, 76-96).
template <unsigned F>
__device__ __forceinline__ float analytic_t(KP p, const FObj& ob, int i, F3 o, F3 d) {
  F3 ro, rd;
  to_object<F>(p, ob, i, o, d, ro, rd);
  // without spheres and boxes in the scene every analytic object is a plane
  if (!(F & (F_SPHERE | F_BOX)) || ob.type == GEOM_PLANE) return plane(ro, rd);
  if ((F & F_SPHERE) && ob.type == GEOM_SPHERE) return sphere(ob.r, ro, rd);
  if (F & F_BOX) return aabb(ob.lo, ob.hi, ro, f3(rcp(rd.x), rcp(rd.y), rcp(rd.z)));
  return -finf();
}

// analytic_t for S rays against one object: the object's transform kind
// and type are dispatched once (uniform branches) with the S rays inside
// each case — called per ray, the dispatch and the object's record loads
// were repeated for every ray (C2's batches: ~20 scalar instructions per ray
// and object on the CU's busiest pipe). Same arithmetic per ray as
// analytic_t (bit-identical t); body(k, t) consumes ray k's t at once, and a
// scheduling barrier between rays keeps their temporaries from overlapping
// (interleaved, the S rays' transforms spilled).
template <unsigned F, int S, class Body>
__device__ __forceinline__ void analytic_t_batch(KP p, const FObj& ob, int i, const F3 (&o)[S], const F3 (&d)[S],
                                                 Body&& body) {
#ifdef RTMI_PER_RAY_DISPATCH  // diagnostic A/B: the dispatch per ray
#pragma unroll
  for (int k = 0; k < S; ++k) body(k, analytic_t<F>(p, ob, i, o[k], d[k]));
  return;
#endif
  auto cases = [&](auto general) {
    constexpr bool G = decltype(general)::value;
    auto xform = [&](int k, F3& ro, F3& rd) {
      if constexpr (G) {
        const RT_CONST FObjX& x = at(p->objx, i);
        const float* m = x.w2o;
        ro = f3(__builtin_fmaf(m[0], o[k].x, __builtin_fmaf(m[3], o[k].y, __builtin_fmaf(m[6], o[k].z, m[9]))),
                __builtin_fmaf(m[1], o[k].x, __builtin_fmaf(m[4], o[k].y, __builtin_fmaf(m[7], o[k].z, m[10]))),
                __builtin_fmaf(m[2], o[k].x, __builtin_fmaf(m[5], o[k].y, __builtin_fmaf(m[8], o[k].z, m[11]))));
        rd = f3(__builtin_fmaf(m[0], d[k].x, __builtin_fmaf(m[3], d[k].y, m[6] * d[k].z)),
                __builtin_fmaf(m[1], d[k].x, __builtin_fmaf(m[4], d[k].y, m[7] * d[k].z)),
                __builtin_fmaf(m[2], d[k].x, __builtin_fmaf(m[5], d[k].y, m[8] * d[k].z)));
      } else {
        ro = f3(o[k].x + ob.t[0], o[k].y + ob.t[1], o[k].z + ob.t[2]);
        rd = d[k];
      }
    };
    if (!(F & (F_SPHERE | F_BOX)) || ob.type == GEOM_PLANE) {
#pragma unroll
      for (int k = 0; k < S; ++k) {
        F3 ro, rd;
        xform(k, ro, rd);
        body(k, plane(ro, rd));
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if ((F & F_SPHERE) && ob.type == GEOM_SPHERE) {
#pragma unroll
      for (int k = 0; k < S; ++k) {
        F3 ro, rd;
        xform(k, ro, rd);
        body(k, sphere(ob.r, ro, rd));
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if (F & F_BOX) {
#pragma unroll
      for (int k = 0; k < S; ++k) {
        F3 ro, rd;
        xform(k, ro, rd);
        body(k, aabb(ob.lo, ob.hi, ro, f3(rcp(rd.x), rcp(rd.y), rcp(rd.z))));
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int k = 0; k < S; ++k) body(k, -finf());
    }
  };
  if ((F & F_XF_GENERAL) && ob.xf == XF_GENERAL)
    cases(Bool<true>{});
  else
    cases(Bool<false>{});
}

// trace (renderer.nim:47-67): linear closest hit over the objects in order;
// an object counts as a hit only when it beats the running minimum.
//
// Shadow rays only need (a) whether any object is hit below tmax and (b) the
// reference's hit count, in which an object after the mesh is counted only if
// its t beats the mesh's closest t. So once a lane has found a mesh hit at
// t <= stop = min t of the analytic objects after the mesh, every later
// comparison is decided and the lane retires: exact, not an approximation.
// Applied when the scene has exactly one mesh object (p->shadow_mesh); stop =
// min t >= 0 of the analytic objects after the mesh.
// pix: the camera ray's pixel index (y * width + x; -1 for other rays),
// light: the shadow ray's light (-1 for other rays); they select the bins.
// The search of the mesh's faces for the lanes that passed the AABB gate
// (part): the shadow early exit's stop distance, the binned lists, then the
// BVH for the lanes no bin served. Returns the best (t, face) key (key0 = the
// entry key when nothing closer was found).
template <bool COUNT, unsigned F>
__device__ __forceinline__ unsigned long long mesh_search(KP p, const FObj& ob, int i, F3 o, F3 d, F3 ro, F3 rd,
                                                          SlabRay sr, bool part, float tb, bool shadow, bool early,
                                                          int bin, const int32_t* boff, const int32_t* bent,
                                                          bool nohit, int light, Stats32& ws) {
  const bool ex = early && i == p->shadow_mesh;
  const char* lb = shadow ? lrec_of(p, light) : nullptr;  // distant-light shadow rays: LTri records
  float stop = -1.0f;
  if (ex) {
    RT_STAMP(t_st0);
    stop = finf();
    for (int j = i + 1; j < p->nobj; ++j) {
      const float tj = analytic_t<F>(p, at(p->objs, j), j, o, d);
      stop = tj >= 0.0f ? fminf(stop, tj) : stop;
    }
#if RTMI_STAMPS == 2
    { RT_STAMP(t_st1); RT_ACC(7, t_st0, t_st1); }
#endif
  }
  // search state of the lanes that enter: the best (t, face) key and
  // the culling limit; a lane retires (early exit) on a FOUND hit
  // with t <= stop, so stop is clamped to the float just below the
  // initial limit (tb > 0; for tb == 0 the bit pattern wraps to NaN,
  // fminf keeps stop, and nothing is acceptable)
  float tc = part ? tb : -1.0f;
  stop = fminf(stop, __uint_as_float(__float_as_uint(tb) - 1u));
  const unsigned long long key0 = part ? tkey(tb, 0u) : 0ull;
  unsigned long long key = key0;
  // shadow rays: the light-grid cell (after the gate: the cell
  // costs more than the gate, which already sends most waves away)
  if ((F & F_MESH) && shadow && p->grids && light >= 0 && p->grids[light].gu > 0) {
    const RT_CONST LightGrid& G = cp(p->grids)[light];
    const float gu = __builtin_fmaf(ro.x, G.e1[0], __builtin_fmaf(ro.y, G.e1[1], ro.z * G.e1[2]));
    const float gv = __builtin_fmaf(ro.x, G.e2[0], __builtin_fmaf(ro.y, G.e2[1], ro.z * G.e2[2]));
    const float fu = (gu - G.u0) * G.inv_h, fv = (gv - G.v0) * G.inv_h;
    const bool safe = fmaxf(fmaxf(fabsf(ro.x), fabsf(ro.y)), fabsf(ro.z)) <= G.rmax;
    const bool on = fu >= 0.0f && fu < (float)G.gu && fv >= 0.0f && fv < (float)G.gv;
    bin = safe && on ? G.off_base + (int)fv * G.gu + (int)fu : -1;
    nohit = safe && !on;
    boff = p->grid_off;
    bent = p->grid_ent + G.ent_base;
  }
  if (bent) {  // up to 4 distinct bins per wave; lanes left over take the BVH
    unsigned long long todo = bal(part && bin >= 0), ovf = 0ull;
    for (int it = 0; it < 4 && todo != 0ull; ++it) {
      const int kb = __builtin_amdgcn_readlane(bin, (int)__builtin_ctzll(todo));
      const unsigned long long mk = bal(bin == kb);
      todo &= ~mk;
      if (boff) {  // a light-grid cell
        list_search<COUNT>(p, bent, cp(boff)[kb], cp(boff)[kb + 1], ro, rd, ex, stop, key, tc, ws, lb);
      } else {     // a pixel list (rt_frame.h slots); past its slots the BVH serves the pixel
        const int n = (int)(at(p->pix_cnt, kb) & kPixCount), b = kb << p->slot_lg;
        if (n > (1 << p->slot_lg)) ovf |= mk;
        else list_search<COUNT>(p, bent, b, b + n, ro, rd, ex, stop, key, tc, ws, lb);
      }
    }
    // done: binned lanes (their bin was searched) and lanes off the grid
    tc = (lane_in(todo | ovf) || !(bin >= 0 || nohit)) ? tc : -1.0f;
  }
  traverse<COUNT>(p, ob.root, ro, rd, sr, ex, stop, key, tc, ws, lb);
  return key;
}


template <bool COUNT, unsigned F>
__device__ __forceinline__ Hit trace(KP p, F3 o, F3 d, float tmax, bool active, bool shadow, int pix, int light,
                                     Stats32& ws, bool no_mesh = false) {
  RT_STAMP(t_trace0);
  Hit h{-1, -1, tmax};
  const bool early = (F & F_MESH) && shadow && p->shadow_mesh >= 0;
#if RTMI_FCMP_MASKS
  const unsigned long long actm = bal(active);
#endif
  // Object bins (scenes of 4..64 objects, rt_bins.h): the objects the wave's
  // bins list, in scene order; an object no bin lists cannot be hit (it
  // would add nothing to the closest hit or the hit count). Up to 4 distinct
  // bins per wave, otherwise every object.
  // Compiled for scenes with spheres or boxes only: mesh + plane scenes keep
  // the plain object loop (C3: the mask loop cost 27 % there).
  constexpr bool kObjBins = (F & (F_SPHERE | F_BOX)) != 0;
  const int nobj = p->nobj;
  unsigned long long omask = nobj >= 64 ? ~0ull : ((1ull << nobj) - 1ull);
  if (!kObjBins) {
  } else if (!shadow && p->obj_pix && pix >= 0) {  // camera rays: the wave's pixels
    unsigned long long todo = bal(active && pix >= 0), m = 0ull;
    for (int it = 0; it < 4 && todo != 0ull; ++it) {
      const int kp = __builtin_amdgcn_readlane(pix, (int)__builtin_ctzll(todo));
      todo &= ~bal(pix == kp);
      m |= cp(p->obj_pix)[kp];
    }
    omask = todo == 0ull ? m : omask;
  } else if (shadow && p->obj_grids && light >= 0 && p->obj_grids[light].gu > 0) {  // distant light: cells
    const RT_CONST LightGrid& G = cp(p->obj_grids)[light];
    const float gu = __builtin_fmaf(o.x, G.e1[0], __builtin_fmaf(o.y, G.e1[1], o.z * G.e1[2]));
    const float gv = __builtin_fmaf(o.x, G.e2[0], __builtin_fmaf(o.y, G.e2[1], o.z * G.e2[2]));
    const float fu = (gu - G.u0) * G.inv_h, fv = (gv - G.v0) * G.inv_h;
    const bool safe = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z)) <= G.rmax;
    const bool on = fu >= 0.0f && fu < (float)G.gu && fv >= 0.0f && fv < (float)G.gv;
    const int cell = on ? (int)fv * G.gu + (int)fu : -1;
    unsigned long long m = p->obj_off_grid;
    unsigned long long todo = bal(active && safe && on);
    for (int it = 0; it < 4 && todo != 0ull; ++it) {
      const int kc = __builtin_amdgcn_readlane(cell, (int)__builtin_ctzll(todo));
      todo &= ~bal(cell == kc);
      m |= cp(p->obj_grid_mask)[G.off_base + kc];
    }
    omask = (todo == 0ull && bal(active && !safe) == 0ull) ? m : omask;
  }
  auto visit = [&](const int i) {
    // the mesh skipped outright (no record fetch, no hit-mask work)
    if ((F & F_MESH) && no_mesh && i == p->shadow_mesh) return;
    const FObj ob = at(p->objs, i);
    float t;
    int tri = -1;
    if (!(F & F_MESH) || ob.type != GEOM_MESH) {
      t = analytic_t<F>(p, ob, i, o, d);
    } else {
      RT_STAMP(t_g0);
      F3 ro, rd;
      to_object<F>(p, ob, i, o, d, ro, rd);
      // Coherent families search the faces binned for them (rt_bins.h)
      // instead of the BVH: camera rays by pixel (pix: this lane's pixel
      // index, -1 for other rays), shadow rays to a distant light by
      // light-grid cell. A lane whose bin is empty, or that is off the grid,
      // can hit no face. When the caller knows that no lane can hit the mesh
      // (no_mesh: a one-pixel wave whose pixel list is empty, or whose
      // pixel's shadow skip bit for this light is set) the mesh is skipped
      // before the AABB gate (the gate's verdict cannot matter).
      int bin = -1;                        // this lane's bin, -1: none
      const int32_t* boff = nullptr;       // light-grid cells: CSR offsets; pixel lists: slots (boff == nullptr)
      const int32_t* bent = nullptr;
      bool nohit = false;                  // off every listed face
      if ((F & F_MESH) && !shadow && p->pix_slots && pix >= 0) {
        bin = pix;
        bent = p->pix_slots;
      }
      // no_mesh (wave-uniform, the caller's pixel record): no lane can hit the mesh
      const bool skip = no_mesh;
      if (skip) {
        t = -finf();
      } else {
        // TriangleMesh.intersect (geom.nim:339-358): a ray starting inside
        // the mesh AABB misses (entry t < 0); otherwise the closest face.
        // The AABB and the root ride in the object record (no dependent
        // FMesh fetch); the gate uses the traversal's slab form of the ray
        // (built here, not hoisted to the trace's entry by the compiler:
        // camera waves over an empty pixel list never need it).
        F3 rdl = rd;
        asm volatile("" : "+v"(rdl.x), "+v"(rdl.y), "+v"(rdl.z));
        const SlabRay sr = slab_ray(ro, rdl);
        const float ax = __builtin_fmaf(ob.lo[0], sr.ni.x, -sr.oi.x), bx = __builtin_fmaf(ob.hi[0], sr.ni.x, -sr.oi.x);
        const float ay = __builtin_fmaf(ob.lo[1], sr.ni.y, -sr.oi.y), by = __builtin_fmaf(ob.hi[1], sr.ni.y, -sr.oi.y);
        const float az = __builtin_fmaf(ob.lo[2], sr.ni.z, -sr.oi.z), bz = __builtin_fmaf(ob.hi[2], sr.ni.z, -sr.oi.z);
        const float gmin = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
        const float gmax = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz)) * 1.00000024f;
        const bool in = gmin <= gmax && gmin >= 0.0f;
        const bool part = active && in;
        float tb = h.t;
        int best = -1;
#if RTMI_STAMPS == 2
        { RT_STAMP(t_g1); RT_ACC(8, t_g0, t_g1); }
#endif
        // shadow early exit (above): stop is only computed when some lane of
        // the wave enters the mesh
        if (ob.root >= 0 && bal(part) != 0ull) {
          const unsigned long long key0 = part ? tkey(tb, 0u) : 0ull;
          const unsigned long long key = mesh_search<COUNT, F>(p, ob, i, o, d, ro, rd, sr, part, tb, shadow, early,
                                                               bin, boff, bent, nohit, light, ws);
          if (key != key0) {
            tb = __uint_as_float((unsigned int)(key >> 32));
            best = (int)(unsigned int)key;
          }
        }
        t = !in ? -finf() : (best >= 0 ? tb : finf());
        tri = best;
      }
    }
#if RTMI_FCMP_MASKS
    const unsigned long long um = m_ge(t, 0.0f) & m_lt(t, h.t) & actm;
    ws.v[STAT_HITS] += pc(um);
    const bool upd = lane_in(um);
#else
    const bool upd = active && t >= 0.0f && t < h.t;
    ws.v[STAT_HITS] += pc(bal(upd));
#endif
    if (upd) {
      h.t = t;
      h.obj = i;
      h.tri = tri;
    }
  };
  if constexpr (kObjBins) {
    for (int base = 0; base < nobj; base += 64) {
      unsigned long long om = base == 0 ? omask : (nobj - base >= 64 ? ~0ull : ((1ull << (nobj - base)) - 1ull));
      while (om != 0ull) {
        const int i = base + (int)__builtin_ctzll(om);
        om &= om - 1ull;
        visit(i);
      }
    }
  } else {
    for (int i = 0; i < nobj; ++i) visit(i);
  }
#ifdef RTMI_STAMPS
  { RT_STAMP(t_trace1); RT_ACC(6, t_trace0, t_trace1); }
#endif
  return h;
}

// normal(*) (geom.nim:361-379) for analytic geometry, object space.
template <unsigned F>
__device__ __forceinline__ F3 analytic_normal(const FObj& ob, F3 ho) {
  if ((F & F_SPHERE) && ob.type == GEOM_SPHERE) {
    const float r = rsq(dot3(ho, ho));
    return f3(ho.x * r, ho.y * r, ho.z * r);
  }
  if ((F & F_BOX) && ob.type == GEOM_BOX) {
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

// Per-lane LDS scratch of the shading loop, laid out [slot][lane] so a
// wave's access to one slot touches 64 consecutive dwords (no bank
// conflicts). Parking the reflected ray and the hit point here instead of in
// VGPRs takes them out of the register peak, which sits inside the
// shadow-ray traversal (DESIGN.md "Occupancy").
enum : int { LDS_RO = 0, LDS_RD = 3, LDS_HW = 6, LDS_ALB = 9, kLdsSlots = 12 };
// An LDS-typed pointer: 32-bit addresses with the slot offsets folded into
// the ds_* immediates (a generic float* here became a 64-bit flat address
// per slot, hoisted and pinned in VGPRs).
#if defined(__HIP_DEVICE_COMPILE__)
using LdsF = __attribute__((address_space(3))) float;
#else
using LdsF = float;
#endif

// Radiance accumulator of the lane's current pixel samples. Kept in VGPRs:
// LDS float atomics (ds_add_f32) measured ~50 % slower on C3 and a plain
// LDS read-modify-write no faster than the three registers.
struct Acc {
  F3 v;
};
__device__ __forceinline__ void acc_add3(Acc& a, float x, float y, float z) {
  a.v = f3(a.v.x + x, a.v.y + y, a.v.z + z);
}
// A shading level's radiance, in the reference's grouping (shade() sums the
// lights' shadeDiffuse terms, renderer.nim:93-104, and calcPixel adds each
// sample's colour, renderer.nim:149-157): per light E += ci * ndl (one FMA
// per channel), then the level adds albedo/pi * weight * E — rounded the same
// way by every instance of the sample loop (no contraction choices left to
// the compiler), so the batched lean samples below and the one-sample loop
// give bit-identical pixels.
__device__ __forceinline__ void irr_add(F3& e, const float* ci, float ndl) {
  e = f3(__builtin_fmaf(ci[0], ndl, e.x), __builtin_fmaf(ci[1], ndl, e.y), __builtin_fmaf(ci[2], ndl, e.z));
}
// A product the compiler may not fuse into a later add (-ffp-contract=fast
// contracts HIP's __fmul_rn, a plain `*`, wherever the add happens to be
// visible): the empty asm makes the product opaque, at no instruction cost.
__device__ __forceinline__ float mul_nc(float a, float b) {
  float r = a * b;
  asm("" : "+v"(r));
  return r;
}
__device__ __forceinline__ F3 mul3(F3 a, F3 b) { return f3(mul_nc(a.x, b.x), mul_nc(a.y, b.y), mul_nc(a.z, b.z)); }
// volatile: the value must really leave the registers (no store-to-load
// forwarding across the light loop)
__device__ __forceinline__ void lds_put3(LdsF* ls, int slot, F3 v) {
  volatile LdsF* q = ls;
  q[(slot + 0) * 64] = v.x;
  q[(slot + 1) * 64] = v.y;
  q[(slot + 2) * 64] = v.z;
}
__device__ __forceinline__ F3 lds_get3(LdsF* ls, int slot) {
  volatile LdsF* q = ls;
  return f3(q[(slot + 0) * 64], q[(slot + 1) * 64], q[(slot + 2) * 64]);
}

// One shading level of renderer.nim's shade (renderer.nim:71-127 at one
// recursion depth) for the wave's `act` lanes, at forward weight w:
//  * renderer.nim:94-101: one shadow ray per light from hitW + N*bias; the
//    light's shadeDiffuse term (shader.nim:12-17) is added when it misses.
//  * renderer.nim:104-124: reflection > 0 and depth <= maxRayDepth traces
//    r = i - 2 (n.i) n from hitW + r*bias; the level's local light is
//    weighted (1 - reflection), the reflected colour reflection.
// v: the level's radiance of this lane (background x w on a miss, the
// weighted local light on a hit); reflect / refl: whether the lane reflects
// (its reflected ray parked in LDS at LDS_RO / LDS_RD) and the hit's
// Material.reflection (0 without a hit).
// pix: the sample's pixel index (y * width + x) for the camera ray's bins;
// pinfo: the wave's pixel record (FastParams.pix_info) when the wave holds
// one pixel, else kPixCount (nothing known).
template <bool COUNT, unsigned F, bool LEAN = false>
__device__ __forceinline__ void shade_level(KP& p, F3 o, F3 d, bool act, int lev, int depth, float w, int pix,
                                            unsigned pinfo, LdsF* ls, F3& v, bool& reflect, float& refl_out,
                                            Stats32& ws) {
  v = f3(0.0f, 0.0f, 0.0f);
  const Hit hit = trace<COUNT, F>(p, o, d, finf(), act, false, lev == 0 ? pix : -1, -1, ws,
                                  lev == 0 && (LEAN || (pinfo & kPixCount) == 0u));
  if (act && hit.obj < 0) v = f3(mul_nc(w, p->bg[0]), mul_nc(w, p->bg[1]), mul_nc(w, p->bg[2]));
  const bool lit = act && hit.obj >= 0;
  const F3 hw = f3(__builtin_fmaf(d.x, hit.t, o.x), __builtin_fmaf(d.y, hit.t, o.y), __builtin_fmaf(d.z, hit.t, o.z));
  F3 N = f3(0.0f, 0.0f, 0.0f);
  F3 alb = f3(0.0f, 0.0f, 0.0f);
  float refl = 0.0f;
  unsigned long long pending = bal(lit);
  while (pending) {  // one pass per distinct object hit by the wave
    const int lead = (int)__builtin_ctzll(pending);
    const int oi = __builtin_amdgcn_readlane(hit.obj, lead);
    // `mine` compares against an opaque copy: knowing hit.obj == oi inside
    // the branch, the compiler would otherwise address the object's
    // uniform records through the per-lane hit.obj (vector loads on the
    // sample's critical path instead of scalar loads)
    int oi_cmp = oi;
    asm volatile("" : "+s"(oi_cmp));
    const bool mine = lit && hit.obj == oi_cmp;
    pending &= ~bal(mine);
    const FObj ob = at(p->objs, oi);
    const RT_CONST FObjX& ox = at(p->objx, oi);
    const F3 oalb = f3(ox.albedo_pi[0], ox.albedo_pi[1], ox.albedo_pi[2]);
    const float orefl = ox.refl;
    const int nbase = ox.normal_base;
    if (mine) {
      F3 n;
      if ((F & F_MESH) && ob.type == GEOM_MESH) {
        const float* fn = p->normals + 3 * (size_t)(nbase + hit.tri);
        n = f3(fn[0], fn[1], fn[2]);
      } else {
        F3 ho, unused;
        to_object<F>(p, ob, oi, hw, f3(0.0f, 0.0f, 0.0f), ho, unused);
        n = analytic_normal<F>(ob, ho);
      }
      if ((F & F_XF_GENERAL) && ob.xf == XF_GENERAL) {  // object_to_world * n, not re-normalised
        const float* m = ox.o2w;
        N = f3(__builtin_fmaf(m[0], n.x, __builtin_fmaf(m[3], n.y, m[6] * n.z)),
               __builtin_fmaf(m[1], n.x, __builtin_fmaf(m[4], n.y, m[7] * n.z)),
               __builtin_fmaf(m[2], n.x, __builtin_fmaf(m[5], n.y, m[8] * n.z)));
      } else {
        N = n;
      }
      alb = oalb;
      refl = orefl;
    }
  }
  reflect = (F & F_REFLECT) && lit && refl > 0.0f && depth <= p->max_depth;
  refl_out = refl;
  const float wl = reflect ? w * (1.0f - refl) : w;
  // albedo/pi * weight waits in LDS across the light loop (the loop's
  // register peak sits inside the shadow traversal); the lights' terms
  // are summed into E first (irr_add)
  lds_put3(ls, LDS_ALB, f3(alb.x * wl, alb.y * wl, alb.z * wl));
  F3 E = f3(0.0f, 0.0f, 0.0f);
  if (F & F_REFLECT) ws.v[STAT_REFL] += pc(bal(reflect));
  if ((F & F_REFLECT) && bal(reflect)) {  // park the reflected ray (renderer.nim:109-118)
    if (reflect) {
      const float ndi = 2.0f * dot3(N, d);
      const F3 rd = f3(d.x - N.x * ndi, d.y - N.y * ndi, d.z - N.z * ndi);
      lds_put3(ls, LDS_RO, f3(__builtin_fmaf(rd.x, p->bias, hw.x), __builtin_fmaf(rd.y, p->bias, hw.y),
                              __builtin_fmaf(rd.z, p->bias, hw.z)));
      lds_put3(ls, LDS_RD, rd);
    }
  }
  const F3 so = f3(__builtin_fmaf(N.x, p->bias, hw.x), __builtin_fmaf(N.y, p->bias, hw.y),
                   __builtin_fmaf(N.z, p->bias, hw.z));
  if ((F & F_POINT) && p->has_point_light) lds_put3(ls, LDS_HW, hw);
  // no lane shaded a hit (the sky): no shadow rays at all
  const int nl = bal(lit) != 0ull ? p->nlight : 0;
  // shadow skips of the wave's pixel (camera hits only): bit li set = no
  // shadow ray to light li can meet the mesh
  const unsigned skipw = lev == 0 ? pinfo >> 24 : 0u;
  // two instances of the light loop: with every light's skip bit set the
  // shadow traces are compiled without the mesh search (C3: most waves),
  // which the register allocation and scheduling of the loop feel even
  // when the search is skipped at run time
  auto light_loop = [&](auto lean) {
    constexpr bool kLean = decltype(lean)::value;
    for (int li = 0; li < nl; ++li) {
      if (!kLean) p = params();
      const FLight L = at(p->lights, li);
      F3 sd;
      float dist, k = 1.0f;
      if ((F & F_POINT) && L.type == LIGHT_POINT) {  // light.nim:52-62
        const F3 h = lds_get3(ls, LDS_HW);
        const F3 lv = f3(h.x - L.v[0], h.y - L.v[1], h.z - L.v[2]);
        const float r2 = dot3(lv, lv);
        const float rr = rsq(r2);
        sd = f3(-lv.x * rr, -lv.y * rr, -lv.z * rr);
        k = rcp(12.566370614359172f * r2);
        dist = r2 * rr;
      } else {  // light.nim:46-50
        sd = f3(-L.v[0], -L.v[1], -L.v[2]);
        dist = finf();
      }
      ws.v[STAT_SHADOW] += pc(bal(lit));
      const Hit sh = trace<COUNT, F>(p, so, sd, dist, lit, true, -1, li, ws,
                                     kLean || (li < 8 && ((skipw >> li) & 1u) != 0u));
      if (lit && sh.obj < 0) irr_add(E, L.ci, fmaxf(dot3(N, sd), 0.0f) * k);  // shadeDiffuse (shader.nim:12-17)
    }
  };
  if (LEAN || ((F & F_MESH) && nl > 0 && nl <= 8 && skipw == (1u << nl) - 1u))
    light_loop(Bool<true>{});
  else
    light_loop(Bool<false>{});
  if (lit) v = mul3(lds_get3(ls, LDS_ALB), E);
}

// One camera sample: trace + shade (renderer.nim:71-127), reflections as a
// loop of levels with forward weights; each level's radiance is added into
// `acc` in level order.
template <bool COUNT, unsigned F, bool LEAN = false>
__device__ __forceinline__ void shade_path(KP p, F3 o, F3 d, bool active, int pix, unsigned pinfo, LdsF* ls,
                                           Acc& acc, Stats32& ws) {
  bool act = active;
  int depth = 1;
  float w = 1.0f;
  for (int lev = 0; lev < ((F & F_REFLECT) ? kMaxShadeLevels : 1); ++lev) {
    if (LEAN == 0) p = params();
    if (bal(act) == 0ull) break;
    F3 v;
    bool reflect;
    float refl;
    shade_level<COUNT, F, LEAN>(p, o, d, act, lev, depth, w, pix, pinfo, ls, v, reflect, refl, ws);
    if (act) acc_add3(acc, v.x, v.y, v.z);
    // every lane reloads (lanes that do not reflect go inactive): o and d
    // are then dead across the light loop instead of carried for them
    if ((F & F_REFLECT) && bal(reflect)) {
      o = lds_get3(ls, LDS_RO);
      d = lds_get3(ls, LDS_RD);
    }
    w = w * refl;
    ++depth;
    act = reflect;
  }
}

#ifndef RTMI_QUEUE_AHEAD
#define RTMI_QUEUE_AHEAD 1
#endif

// Occupancy target (k_render_fast, k_render_wave). Fewer resident waves
// buy registers: the instances whose loops spilled at 8 waves/SIMD run at 5
// (<= 96 VGPRs): meshes with point lights or reflection (mesh-mix 1080p/64
// spp: 8 -> 5 waves 4.20 -> 3.44 ms) and the analytic scenes, whose
// object-binned batches carry 4 samples per lane (C2 0.98 -> 0.85 ms with the
// per-object dispatch below; spheres-* unchanged). The mesh + plane instance
// runs at RTMI_MESH_WAVES = 7 (<= 72 VGPRs; 8 / 7 / 6 waves, 1080p: bunny
// 256 spp one-kernel 2.36 / 2.09 / 2.18 ms, bunny 4 spp 0.334 / 0.308 /
// 0.320, two-meshes 64 spp 3.11 / 2.92 / 3.00; round 1's 8-wave choice
// predates the pixel records and batched lean paths).
#ifndef RTMI_MESH_WAVES
#define RTMI_MESH_WAVES 7
#endif
// Subsets that would spill more than 8 VGPRs at their family's default run
// at the highest occupancy that does not (rt_occupancy.h, generated by
// tools/occupancy_table.py from the compiler's resource usage; VERDICT r4:
// the mesh subsets with spheres / boxes / rotations spilled up to 71 VGPRs).
// The generator itself compiles with RTMI_NO_OCC_TABLE.
template <unsigned F>
constexpr unsigned subset_index() {
  return (F & 1u) | (F & 2u) | ((F & 8u) ? 4u : 0u) | ((F & 16u) ? 8u : 0u) | ((F & 32u) ? 16u : 0u) |
         ((F & 64u) ? 32u : 0u) | ((F & 128u) ? 64u : 0u);
}
template <unsigned F>
constexpr unsigned occ_table(const unsigned char (&t)[128], unsigned dflt) {
#ifdef RTMI_NO_OCC_TABLE
  (void)t;
  return dflt;
#else
  return t[subset_index<F>()] ? t[subset_index<F>()] : dflt;
#endif
}
#ifndef RTMI_ANALYTIC_WAVES
#define RTMI_ANALYTIC_WAVES 5  // the other subsets (analytic scenes, point lights, reflection)
#endif
template <unsigned F>
constexpr unsigned waves_per_eu() {
#ifdef RTMI_WAVES_PER_EU
  return RTMI_WAVES_PER_EU;
#else
  return occ_table<F>(kOcc_fast, ((F & F_MESH) && !(F & (F_POINT | F_REFLECT))) ? RTMI_MESH_WAVES
                                                                                 : RTMI_ANALYTIC_WAVES);
#endif
}
template <unsigned F>
constexpr unsigned wave_waves() {  // k_render_wave
#ifdef RTMI_WAVES_PER_EU
  return RTMI_WAVES_PER_EU;
#else
  return occ_table<F>(kOcc_wave, ((F & F_MESH) && !(F & (F_POINT | F_REFLECT))) ? RTMI_MESH_WAVES : 5u);
#endif
}
#define RTMI_OCC __attribute__((amdgpu_waves_per_eu(waves_per_eu<F>())))
// The lane id from an opaque instruction: values derived from it are
// recomputed inside the loops instead of hoisted to kernel scope, where
// they would stay live (and spill) across the whole sample loop.
__device__ __forceinline__ int lane_id_fresh() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// q = n / dv, r = n - q*dv for 0 <= n < 2^21 and dv >= 1 via the float
// reciprocal (exact: the quotient's fractional part keeps >= 0.5/dv from an
// integer, far above the fp32 product's error); no integer-division sequence.
__device__ __forceinline__ int div_small(int n, int dv, float inv_dv, int& r) {
  const int q = (int)(((float)n + 0.5f) * inv_dv);
  r = n - q * dv;
  return q;
}

// A pixel group's placement: tile (tx x ty pixels, L lanes each, powers of
// two) -> this lane's pixel (x, y), output row and validity.
struct GroupPix {
  int x, y, out_row, sub;
  bool valid;
};
__device__ __forceinline__ GroupPix group_pixel(KP p, int g, int lane) {
  GroupPix r;
  r.sub = lane & (p->lanes_per_px - 1);
  const int pix = lane >> p->log2_lanes;
  const int tpx = pix & (p->tile_x - 1), tpy = pix >> p->log2_tile_x;
  const int gy = (int)(((unsigned long long)(unsigned)g * p->tx_magic) >> p->tx_shift);  // g / tiles_x (scalar)
  const int gx = g - gy * p->tiles_x;
  const int j = gx * p->tile_x + tpx;
  const int k = gy * p->tile_y + tpy;
  r.x = j * p->step;
  r.valid = j < p->ncols && k < p->nrows;
  if (p->mode == 0) {
    r.y = p->y0 + k * p->step;
    r.out_row = r.y;
  } else {  // round-robin bands (rt_render_bands_device)
    int rr;
    const int lb = div_small(k, p->band_h, p->inv_band_h, rr);
    r.y = (lb * p->world + p->rank) * p->band_h + rr;
    r.out_row = k;
    r.valid = r.valid && r.y < p->height;
  }
  if (p->step < p->max_step) {  // progressive refinement skip (renderer.nim:175-178)
    const int mask = p->step * 2 - 1;
    if ((r.x & mask) == 0 && (r.y & mask) == 0) r.valid = false;
  }
  return r;
}

// castPrimaryRay (renderer.nim:31-44) for sample s of the lane's pixel
// (calcPixel's sample table, renderer.nim:144-159): the direction (the
// origin is the camera's, p->cam[0..2]). Camera constants are folded on the
// host: ((2 x r)/w - r) f == (x - w/2) (2 r f / w), exact 0 on the centre
// column / row as the reference's own formula gives there. Every FMA is
// explicit, so all instances of the sample loop round alike. The cx terms
// are innermost: a lane whose samples share a column (akGrid, m | 64) forms
// them once per pixel (k_render_lean1) with the same roundings.
__device__ __forceinline__ F3 camera_ray_dir(KP p, float px, float py) {
  const float cx = (px - p->cam_b) * p->cam_a;
  const float cy = (p->cam_d - py) * p->cam_c;
  const float rl = rsq(__builtin_fmaf(cy, cy, __builtin_fmaf(cx, cx, 1.0f)));
  return f3(__builtin_fmaf(cy, p->cam[6], __builtin_fmaf(cx, p->cam[3], -p->cam[9])) * rl,
            __builtin_fmaf(cy, p->cam[7], __builtin_fmaf(cx, p->cam[4], -p->cam[10])) * rl,
            __builtin_fmaf(cy, p->cam[8], __builtin_fmaf(cx, p->cam[5], -p->cam[11])) * rl);
}

// Sum of a per-lane count over the wave (DPP row sums, then the rows).
__device__ __forceinline__ unsigned wave_sum(unsigned v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);  // row_shr:8 -> lane 15 of each row: its row's sum
  return (unsigned)__builtin_amdgcn_readlane((int)v, 15) + (unsigned)__builtin_amdgcn_readlane((int)v, 31) +
         (unsigned)__builtin_amdgcn_readlane((int)v, 47) + (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}

// Sum of a float over the wave, in lane 63's order-independent-of-data
// sequence (DPP row_shr scans, then row_bcast:15 / :31), returned uniform.
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_add(float v) {
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWS, 0xf, false));
}
// OR of a 32-bit value over the wave (the DPP tree of wave_total; lanes a
// row shift or broadcast does not reach contribute 0, the identity)
template <int CTRL, int ROWS>
__device__ __forceinline__ unsigned dpp_or(unsigned v) {
  return v | (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, false);
}
__device__ __forceinline__ unsigned wave_or(unsigned v) {
  v = dpp_or<0x111, 0xf>(v);
  v = dpp_or<0x112, 0xf>(v);
  v = dpp_or<0x114, 0xf>(v);
  v = dpp_or<0x118, 0xf>(v);
  v = dpp_or<0x142, 0xa>(v);
  v = dpp_or<0x143, 0xc>(v);
  return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ float wave_total(float v) {
  v = dpp_add<0x111, 0xf>(v);  // row_shr:1
  v = dpp_add<0x112, 0xf>(v);  // row_shr:2
  v = dpp_add<0x114, 0xf>(v);  // row_shr:4
  v = dpp_add<0x118, 0xf>(v);  // row_shr:8: lane 15 of each row holds its row's sum
  v = dpp_add<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
  v = dpp_add<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3: lane 63 holds the total
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// The wave's 32-bit Stats counters into its 64-bit LDS totals (lane k adds
// slot k), then cleared.
__device__ __forceinline__ void flush_stats(Stats32& ws, unsigned long long* tot, int lane) {
  unsigned int v = 0u;
#pragma unroll
  for (int k = 0; k < kStatSlots; ++k) v = lane == k ? ws.v[k] : v;
  if (lane < kStatSlots) tot[lane] += v;
#pragma unroll
  for (int k = 0; k < kStatSlots; ++k) ws.v[k] = 0u;
}

template <unsigned F>
__device__ __forceinline__ void camera_pos(KP p, const GroupPix& gp, int s, const LdsF* tb, float& px_out,
                                           float& py_out) {
  float px = (float)gp.x, py = (float)gp.y;
  if (p->aa_kind == 1) {  // grid() sampling.nim:5-18: sample s = (si, sj)
    int si, sj;
    if (p->log2_grid_m >= 0) {
      si = s & (p->grid_m - 1);
      sj = s >> p->log2_grid_m;
    } else {
      sj = div_small(s, p->grid_m, p->sample_step, si);
    }
    px += __builtin_fmaf((float)si, p->sample_step, p->sample_off);
    py += __builtin_fmaf((float)sj, p->sample_step, p->sample_off);
  } else if ((F & F_STOCHASTIC) && p->aa_kind == 2) {  // jitteredGrid (sampling.nim:21-33): no table needed
    double a, b;
    jittered_entry(rng_pixel_key(p->seed, gp.x, gp.y), p->grid_m, s, a, b);
    px += (float)a;
    py += (float)b;
  } else if ((F & F_STOCHASTIC) && tb) {
    const volatile LdsF* t = tb;
    px += t[s];
    py += t[p->spp + s];
  }
  px_out = px;
  py_out = py;
}
template <unsigned F>
__device__ __forceinline__ F3 camera_dir(KP p, const GroupPix& gp, int s, const LdsF* tb) {
  float px, py;
  camera_pos<F>(p, gp, s, tb, px, py);
  return camera_ray_dir(p, px, py);
}

// The object of the lowest pending lane of the lowest pending sample (-1:
// none). A branch per sample: the branch-free form (a readlane per sample,
// scalar selects) measured 5 % slower on C3.
template <int S>
__device__ __forceinline__ int first_pending(const unsigned long long (&pend)[S], const int (&hob)[S]) {
  int oi = -1;
#pragma unroll
  for (int k = S - 1; k >= 0; --k)
    if (pend[k]) oi = __builtin_amdgcn_readlane(hob[k], (int)__builtin_ctzll(pend[k]));
  return oi;
}

// Sample positions of a batch (S samples per lane: iterations it0 .. it0+S-1
// of a one-pixel wave) and their camera-ray directions; akGrid with m a
// power of two (C2-C5) as s = (s & (m-1), s >> log2 m), the sampler decided
// once for the batch.
template <unsigned F, int S>
__device__ __forceinline__ void batch_dirs(KP p, const GroupPix& gp, int it0, const LdsF* tb, F3 (&d)[S],
                                           bool (&sv)[S]) {
  float px[S], py[S];
  // validity without short-circuit branches (a per-lane && became an
  // exec-mask branch with the argument load inside, per sample)
  const int spp = p->spp;
  const int L = p->lanes_per_px;  // 64: one-pixel waves; 16: object-binned batches of 4 pixels
  if (p->aa_kind == 1 && p->log2_grid_m >= 0 && p->log2_grid_m <= p->log2_lanes) {
    // m divides L: sample s = it * L + sub keeps the lane's column
    // s & (m-1) = sub & (m-1) in every iteration — px (and the camera ray's
    // cx) once per batch, the same values as per sample
    const int mm = p->grid_m - 1, lg = p->log2_grid_m;
    const float st = p->sample_step, of = p->sample_off;
    const float pxl = (float)gp.x + __builtin_fmaf((float)(gp.sub & mm), st, of);
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const int s = (it0 + k) * L + gp.sub;
      sv[k] = gp.valid & (s < spp);
      px[k] = pxl;
      py[k] = (float)gp.y + __builtin_fmaf((float)(s >> lg), st, of);
    }
  } else if (p->aa_kind == 1 && p->log2_grid_m >= 0) {
    const int mm = p->grid_m - 1, lg = p->log2_grid_m;
    const float st = p->sample_step, of = p->sample_off;
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const int s = (it0 + k) * L + gp.sub;
      sv[k] = gp.valid & (s < spp);
      px[k] = (float)gp.x + __builtin_fmaf((float)(s & mm), st, of);
      py[k] = (float)gp.y + __builtin_fmaf((float)(s >> lg), st, of);
    }
  } else {
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const int s = (it0 + k) * L + gp.sub;
      sv[k] = gp.valid & (s < spp);
      camera_pos<F>(p, gp, s < spp ? s : 0, tb, px[k], py[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < S; ++k) d[k] = camera_ray_dir(p, px[k], py[k]);
}

// Lean pixels, kLeanBatch samples per lane at once. A lean pixel (one-pixel
// wave; its pixel list is empty and every light is a distant light whose
// shadow skip bit is set, no reflection: FastParams.pix_info) never touches
// the mesh, so its samples only visit the analytic objects. The per-sample
// loop pays the scalar work of every object visit (record loads, type
// dispatch, loop control, hit-count popcounts: the CU's one scalar unit,
// shared by its 32 resident waves, is the kernel's busiest pipe) once per 64
// rays; here each lane carries kLeanBatch samples through the same object
// and light loops, so that work is paid once per 64 x kLeanBatch rays. Same
// arithmetic per sample as shade_path (camera_dir, analytic_t, the
// irradiance sum), the samples' colours added to the pixel in sample order:
// frames bit-identical to the one-sample loop (tests: binned vs
// RT_FLAG_NO_BINNING, which takes no pixel records).
// trace's hit rule "t >= 0 and t < lim" (renderer.nim:58-62) for a limit lim
// in [+0, +inf] as ONE unsigned compare of the float bits: non-negative
// floats order like their bit patterns, a negative t or a NaN has bits above
// every such lim, and t + 0.0f turns -0.0 (which the rule accepts) into
// +0.0 and leaves every other value as it is. The float form is two compares
// and a scalar AND of their lane masks per ray and object (the batches'
// busiest pipe is the CU's one scalar unit). A sample that takes no part
// holds lim = +0.0, below which nothing lies. RTMI_HIT_UINT=0: the float form.
#ifndef RTMI_HIT_UINT
#define RTMI_HIT_UINT 1
#endif
__device__ __forceinline__ bool hit_below(float t, float lim) {
#if RTMI_HIT_UINT
  return __float_as_uint(t + 0.0f) < __float_as_uint(lim);
#else
  return t >= 0.0f && t < lim;
#endif
}

#ifndef RTMI_LEAN_BATCH
#define RTMI_LEAN_BATCH 4
#endif
constexpr int kLeanBatch = RTMI_LEAN_BATCH;
// OB (object-binned batches, scenes without a mesh: k_render_fast): the
// camera rays visit only the objects of `cmask` (the wave's pixels' object
// masks, rt_bins.h build_object_pixel_masks) and each light's shadow rays
// only those of the light-grid cells their origins fall in — in scene order,
// exactly as trace's object bins (an object no bin lists cannot be hit, so it
// adds nothing to a closest hit or a hit count).
// RTMI_OB_CELLS_JOINT (default 1): an object-binned batch walks the distinct
// light-grid cells of all its samples' shadow origins once (up to 2 S cells,
// then every object), not each sample's cells in turn (up to 4 each). The
// object mask either way holds every object a shadow ray can hit, so frames
// and Stats do not change.
#ifndef RTMI_OB_CELLS_JOINT
#define RTMI_OB_CELLS_JOINT 2
#endif
template <unsigned F, int S = kLeanBatch, bool OB = false>
__device__ __forceinline__ void lean_batch(KP p, const GroupPix& gp, int it0, const LdsF* tb, Acc& acc,
                                           Stats32& ws, unsigned long long cmask = ~0ull) {
  // Branch-free: per-sample predicates are lane masks in SGPRs and every
  // update is a select (v_cndmask), so the samples' code is straight-line
  // VALU (no exec-mask save / restore per sample). A masked-off term adds an
  // exact zero (fma(ci, 0, E) == E, acc + 0 == acc for the non-negative
  // sums), so values equal shade_path's branchy ones bit for bit.
#ifdef RTMI_DIAG_NOSAMPLES
  return;  // diagnostic build only: the work-item overhead without the samples
#endif
  const F3 o = f3(p->cam[0], p->cam[1], p->cam[2]);
  F3 d[S];
  bool sv[S];
  batch_dirs<F, S>(p, gp, it0, tb, d, sv);
  unsigned nprim = 0u;
  // trace (renderer.nim:47-67) of the camera rays over the analytic objects
  // in scene order (the mesh is left out: none of the pixel's rays can hit
  // it). A hit is t >= 0 below the running minimum th; invalid samples start
  // at th = -1, which no t >= 0 is below (so th alone says: -1 invalid,
  // +inf sky, else a hit). Per-lane hit counts (VALU) instead of a mask
  // popcount per sample and object (SALU).
  float th[S];
  int hob[S];
#pragma unroll
  for (int k = 0; k < S; ++k) {
    nprim += pc(bal(sv[k]));
    th[k] = sv[k] ? finf() : (RTMI_HIT_UINT ? 0.0f : -1.0f);  // (hit_below: +0 takes no hit)
    hob[k] = -1;
  }
  ws.v[STAT_PRIMARY] += nprim;
  const int nobj = p->nobj, mesh = p->shadow_mesh;
#ifndef RTMI_LEAN_NOPIN
  // the record arrays' bases pinned in SGPRs for the batch (opaque): the
  // compiler otherwise re-reads them from the kernel arguments before every
  // object / light visit, a dependent scalar load in front of the record's
  const FObj* objs = p->objs;
  const FLight* lights = p->lights;
  asm volatile("" : "+s"(objs), "+s"(lights));
#else
  const FObj* objs = p->objs;
  const FLight* lights = p->lights;
#endif
  unsigned hitl = 0u;
  // the analytic objects in scene order
  // (one loop with a skip test: two index ranges around the mesh measured
  // 2 % slower, the loop body compiled twice)
  auto analytic_objects = [&](auto&& body) {
    for (int i = 0; i < nobj; ++i)
      if (i != mesh) body(i);
  };
  // OB: the objects of a mask in scene order (object bins exist for <= 64 objects)
  auto masked_objects = [&](unsigned long long m, auto&& body) {
    if constexpr (OB) {
      m &= nobj >= 64 ? ~0ull : ((1ull << nobj) - 1ull);
      while (m != 0ull) {
        const int i = (int)__builtin_ctzll(m);
        m &= m - 1ull;
        if (i != mesh) body(i);
      }
    } else {
      (void)m;
      analytic_objects(body);
    }
  };
  F3 oc[S];
#pragma unroll
  for (int k = 0; k < S; ++k) oc[k] = o;
#ifdef RTMI_DIAG_OB_NOCAM
  cmask &= 1ull;  // diagnostic build only (wrong images): camera rays test object 0 alone
#endif
  masked_objects(cmask, [&](const int i) {
    const FObj ob = at(objs, i);
    analytic_t_batch<F, S>(p, ob, i, oc, d, [&](int k, float t) {
      // trace's rule (t >= 0 ? t : inf) < th, as two compares (th <= inf)
      const bool c = hit_below(t, th[k]);
      th[k] = c ? t : th[k];
      hob[k] = c ? i : hob[k];
      hitl += c ? 1u : 0u;
    });
  });
  // shade (renderer.nim:71-127): normals per distinct object hit, the shadow
  // origins hitW + N * bias. A hit has t < inf (it beat the initial limit).
  unsigned long long litm[S], pend[S];
  F3 N[S], so[S];
#pragma unroll
  for (int k = 0; k < S; ++k) {
    litm[k] = bal(hob[k] >= 0);  // (a hit beat th's start: +inf, or +0 for a sample that takes no part)
    pend[k] = litm[k];
    N[k] = f3(0.0f, 0.0f, 0.0f);
    so[k] = f3(__builtin_fmaf(d[k].x, th[k], o.x), __builtin_fmaf(d[k].y, th[k], o.y),
               __builtin_fmaf(d[k].z, th[k], o.z));  // the hit point until N is known
  }
  // every analytic object a plane (the mesh + plane subsets): a plane's
  // normal does not depend on the hit point, so with ONE object hit by the
  // batch's lit samples (the usual ground pixel) N and each light's N.L
  // are wave-uniform — formed once, the same values as per sample
  constexpr bool kPlanesOnly = !(F & (F_SPHERE | F_BOX));
  int nhobj = 0;
  F3 Nu = f3(0.0f, 0.0f, 0.0f), alb_u = f3(0.0f, 0.0f, 0.0f);
#ifdef RTMI_DIAG_OB_NONORMAL
#pragma unroll
  for (int k = 0; k < S; ++k) pend[k] = 0ull;  // diagnostic build only (wrong images): the normal pass's share
#endif
  for (;;) {
    const int oi = first_pending<S>(pend, hob);
    if (oi < 0) break;
    ++nhobj;
    int oi_cmp = oi;
    asm volatile("" : "+s"(oi_cmp));
    const FObj ob = at(objs, oi);
    const RT_CONST FObjX& ox = at(p->objx, oi);
    if constexpr (kPlanesOnly) {
      F3 n = f3(0.0f, 1.0f, 0.0f);  // Plane normal (geom.nim:365-366)
      if ((F & F_XF_GENERAL) && ob.xf == XF_GENERAL) {  // object_to_world * n, not re-normalised
        const float* m = ox.o2w;
        n = f3(__builtin_fmaf(m[0], n.x, __builtin_fmaf(m[3], n.y, m[6] * n.z)),
               __builtin_fmaf(m[1], n.x, __builtin_fmaf(m[4], n.y, m[7] * n.z)),
               __builtin_fmaf(m[2], n.x, __builtin_fmaf(m[5], n.y, m[8] * n.z)));
      }
      Nu = n;
      alb_u = f3(ox.albedo_pi[0], ox.albedo_pi[1], ox.albedo_pi[2]);
#pragma unroll
      for (int k = 0; k < S; ++k) {
        const unsigned long long mine = bal(hob[k] == oi_cmp) & pend[k];
        pend[k] &= ~mine;
        const bool mi = lane_in(mine);
        N[k] = f3(mi ? n.x : N[k].x, mi ? n.y : N[k].y, mi ? n.z : N[k].z);
      }
      continue;
    }
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const unsigned long long mine = bal(hob[k] == oi_cmp) & pend[k];
      pend[k] &= ~mine;
      F3 ho, unused;
      to_object<F>(p, ob, oi, so[k], f3(0.0f, 0.0f, 0.0f), ho, unused);
      F3 n = analytic_normal<F>(ob, ho);
      if ((F & F_XF_GENERAL) && ob.xf == XF_GENERAL) {  // object_to_world * n, not re-normalised
        const float* m = ox.o2w;
        n = f3(__builtin_fmaf(m[0], n.x, __builtin_fmaf(m[3], n.y, m[6] * n.z)),
               __builtin_fmaf(m[1], n.x, __builtin_fmaf(m[4], n.y, m[7] * n.z)),
               __builtin_fmaf(m[2], n.x, __builtin_fmaf(m[5], n.y, m[8] * n.z)));
      }
      const bool mi = lane_in(mine);
      N[k] = f3(mi ? n.x : N[k].x, mi ? n.y : N[k].y, mi ? n.z : N[k].z);
    }
  }
  const bool uni = kPlanesOnly && nhobj == 1;
  const float bias = p->bias;
#pragma unroll
  for (int k = 0; k < S; ++k)
    so[k] = f3(__builtin_fmaf(N[k].x, bias, so[k].x), __builtin_fmaf(N[k].y, bias, so[k].y),
               __builtin_fmaf(N[k].z, bias, so[k].z));
  // one shadow ray per light and lit sample (distant lights only: a point
  // light has no skip bit, so its pixels are never lean)
  F3 E[S];
  unsigned long long anylit = 0ull;
#pragma unroll
  for (int k = 0; k < S; ++k) {
    E[k] = f3(0.0f, 0.0f, 0.0f);
    anylit |= litm[k];
  }
  const int nl = anylit ? p->nlight : 0;
  unsigned nlit = 0u;
#pragma unroll
  for (int k = 0; k < S; ++k) nlit += pc(litm[k]);
  ws.v[STAT_SHADOW] += (unsigned)nl * nlit;
  auto light_loop = [&](auto uniform) {
    constexpr bool U = decltype(uniform)::value;
    for (int li = 0; li < nl; ++li) {
      const FLight L = at(lights, li);
      const F3 sd = f3(-L.v[0], -L.v[1], -L.v[2]);
      float ts[S];  // unlit samples start at 0 (take no part)
#pragma unroll
      for (int k = 0; k < S; ++k) ts[k] = lane_in(litm[k]) ? finf() : 0.0f;
      unsigned long long smask = ~0ull;  // every object
      if constexpr (OB) {
        // the light-grid cells of the lit samples' shadow origins (trace's
        // rule: off the grid -> the unbounded objects; beyond the grid's
        // float32-safe radius, or more than 4 distinct cells -> every object)
        if (p->obj_grids && cp(p->obj_grids)[li].gu > 0) {
          const RT_CONST LightGrid& G = cp(p->obj_grids)[li];
          unsigned long long m = p->obj_off_grid;
          bool every = false;
#if RTMI_OB_CELLS_JOINT == 2
          // every lane loads its samples' cell masks (vector loads, one round
          // trip), ORed over the wave by DPP — instead of one scalar load per
          // distinct cell, each waited for in turn. No cap on the distinct
          // cells: their union is a subset of "every object" and, the masks
          // being conservative, tests every object a ray can hit.
          unsigned long long mine = 0ull;
#pragma unroll
          for (int k = 0; k < S; ++k) {
            const bool lk = lane_in(litm[k]);
            const F3 q = so[k];
            const float gu = __builtin_fmaf(q.x, G.e1[0], __builtin_fmaf(q.y, G.e1[1], q.z * G.e1[2]));
            const float gv = __builtin_fmaf(q.x, G.e2[0], __builtin_fmaf(q.y, G.e2[1], q.z * G.e2[2]));
            const float fu = (gu - G.u0) * G.inv_h, fv = (gv - G.v0) * G.inv_h;
            const bool safe = fmaxf(fmaxf(fabsf(q.x), fabsf(q.y)), fabsf(q.z)) <= G.rmax;
            const bool on = fu >= 0.0f && fu < (float)G.gu && fv >= 0.0f && fv < (float)G.gv;
            if (lk && safe && on) mine |= p->obj_grid_mask[G.off_base + (int)fv * G.gu + (int)fu];
            every = every || bal(lk && !safe) != 0ull;
          }
          m |= ((unsigned long long)wave_or((unsigned)(mine >> 32)) << 32) | wave_or((unsigned)mine);
#elif RTMI_OB_CELLS_JOINT
          // the distinct cells of all S samples' origins, each mask loaded
          // once (the samples of a pixel's lanes mostly share their cells:
          // per sample the same cells were walked S times)
          int cell[S];
          unsigned long long todo[S], left = 0ull;
#pragma unroll
          for (int k = 0; k < S; ++k) {
            const bool lk = lane_in(litm[k]);
            const F3 q = so[k];
            const float gu = __builtin_fmaf(q.x, G.e1[0], __builtin_fmaf(q.y, G.e1[1], q.z * G.e1[2]));
            const float gv = __builtin_fmaf(q.x, G.e2[0], __builtin_fmaf(q.y, G.e2[1], q.z * G.e2[2]));
            const float fu = (gu - G.u0) * G.inv_h, fv = (gv - G.v0) * G.inv_h;
            const bool safe = fmaxf(fmaxf(fabsf(q.x), fabsf(q.y)), fabsf(q.z)) <= G.rmax;
            const bool on = fu >= 0.0f && fu < (float)G.gu && fv >= 0.0f && fv < (float)G.gv;
            cell[k] = on ? (int)fv * G.gu + (int)fu : -1;
            todo[k] = bal(lk && safe && on);
            left |= todo[k];
            every = every || bal(lk && !safe) != 0ull;
          }
          for (int it = 0; it < 2 * S && left != 0ull; ++it) {
            int kc = 0;
#pragma unroll
            for (int k = S - 1; k >= 0; --k)
              if (todo[k]) kc = __builtin_amdgcn_readlane(cell[k], (int)__builtin_ctzll(todo[k]));
            left = 0ull;
#pragma unroll
            for (int k = 0; k < S; ++k) {
              todo[k] &= ~bal(cell[k] == kc);
              left |= todo[k];
            }
            m |= cp(p->obj_grid_mask)[G.off_base + kc];
          }
          every = every || left != 0ull;
#else
#pragma unroll
          for (int k = 0; k < S; ++k) {
            const bool lk = lane_in(litm[k]);
            const F3 q = so[k];
            const float gu = __builtin_fmaf(q.x, G.e1[0], __builtin_fmaf(q.y, G.e1[1], q.z * G.e1[2]));
            const float gv = __builtin_fmaf(q.x, G.e2[0], __builtin_fmaf(q.y, G.e2[1], q.z * G.e2[2]));
            const float fu = (gu - G.u0) * G.inv_h, fv = (gv - G.v0) * G.inv_h;
            const bool safe = fmaxf(fmaxf(fabsf(q.x), fabsf(q.y)), fabsf(q.z)) <= G.rmax;
            const bool on = fu >= 0.0f && fu < (float)G.gu && fv >= 0.0f && fv < (float)G.gv;
            const int cell = on ? (int)fv * G.gu + (int)fu : -1;
            unsigned long long todo = bal(lk && safe && on);
            for (int it = 0; it < 4 && todo != 0ull; ++it) {
              const int kc = __builtin_amdgcn_readlane(cell, (int)__builtin_ctzll(todo));
              todo &= ~bal(cell == kc);
              m |= cp(p->obj_grid_mask)[G.off_base + kc];
            }
            every = every || todo != 0ull || bal(lk && !safe) != 0ull;
          }
#endif
          smask = every ? smask : m;
        }
      }
#ifdef RTMI_DIAG_OB_NOSHADOW
      smask = 0ull;  // diagnostic build only (wrong images): the shadow rays' object tests' share
#endif
      masked_objects(smask, [&](const int i) {
        const FObj ob = at(objs, i);
        if constexpr (kPlanesOnly) {
          // Plane.intersect (geom.nim:240-248) of the parallel shadow rays:
          // the direction's test and reciprocal once (a NaN multiplier for a
          // direction parallel to the plane: no t >= 0, as -inf gives none)
          F3 r0, rdu;
          to_object<F>(p, ob, i, so[0], sd, r0, rdu);
          const float mulp = fabsf(rdu.y) > 1e-6f ? rcp(rdu.y) : __builtin_nanf("");
#pragma unroll
          for (int k = 0; k < S; ++k) {
            F3 ro, rd;
            to_object<F>(p, ob, i, so[k], sd, ro, rd);
            const float t = -ro.y * mulp;
            const bool c = hit_below(t, ts[k]);
            ts[k] = c ? t : ts[k];
            hitl += c ? 1u : 0u;
          }
        } else {
          F3 sdk[S];
#pragma unroll
          for (int k = 0; k < S; ++k) sdk[k] = sd;
          analytic_t_batch<F, S>(p, ob, i, so, sdk, [&](int k, float t) {
            const bool c = hit_below(t, ts[k]);
            ts[k] = c ? t : ts[k];
            hitl += c ? 1u : 0u;
          });
        }
      });
      // unoccluded: shadeDiffuse (shader.nim:12-17)
      const float ndl_u = U ? fmaxf(dot3(Nu, sd), 0.0f) : 0.0f;
#pragma unroll
      for (int k = 0; k < S; ++k) {
        const bool vis = lane_in(litm[k]) && !(ts[k] < finf());
        irr_add(E[k], L.ci, vis ? (U ? ndl_u : fmaxf(dot3(N[k], sd), 0.0f)) : 0.0f);
      }
    }
  };
  if (uni)
    light_loop(Bool<true>{});
  else
    light_loop(Bool<false>{});
  ws.v[STAT_HITS] += wave_sum(hitl);
  // albedo / pi per distinct object hit (one object: from the normal pass),
  // then the samples' colours in order
  if (uni) {
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const F3 a = mul3(alb_u, E[k]);
      const bool mi = lane_in(litm[k]);
      E[k] = f3(mi ? a.x : E[k].x, mi ? a.y : E[k].y, mi ? a.z : E[k].z);
    }
  } else {
#pragma unroll
    for (int k = 0; k < S; ++k) pend[k] = litm[k];
    for (;;) {
      const int oi = first_pending<S>(pend, hob);
      if (oi < 0) break;
      int oi_cmp = oi;
      asm volatile("" : "+s"(oi_cmp));
      const RT_CONST FObjX& ox = at(p->objx, oi);
      const F3 alb = f3(ox.albedo_pi[0], ox.albedo_pi[1], ox.albedo_pi[2]);
#pragma unroll
      for (int k = 0; k < S; ++k) {
        const unsigned long long mine = bal(hob[k] == oi_cmp) & pend[k];
        pend[k] &= ~mine;
        const F3 a = mul3(alb, E[k]);
        const bool mi = lane_in(mine);
        E[k] = f3(mi ? a.x : E[k].x, mi ? a.y : E[k].y, mi ? a.z : E[k].z);
      }
    }
  }
  const F3 bg = f3(p->bg[0], p->bg[1], p->bg[2]);
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const bool lt = lane_in(litm[k]), sky = th[k] == finf();
    const F3 c = f3(lt ? E[k].x : (sky ? bg.x : 0.0f), lt ? E[k].y : (sky ? bg.y : 0.0f),
                    lt ? E[k].z : (sky ? bg.z : 0.0f));
    acc_add3(acc, c.x, c.y, c.z);
  }
}

// tri_test for a ray that only needs the closest t (shadow rays): the best
// t's float bits replace the (t, face) key — a tie never changes t, so t,
// the culling limit tc and "found" follow tri_test's exactly. A lane that
// takes no part holds best = +0.0 (nothing is below it).
template <class TR>
__device__ __forceinline__ void tri_test_t(const TR& T, F3 o, F3 d, float& best, float& tc) {
  const float tx = o.x - T.v0[0], ty = o.y - T.v0[1], tz = o.z - T.v0[2];
  const float cx = __builtin_fmaf(ty, d.z, -tz * d.y);
  const float cy = __builtin_fmaf(tz, d.x, -tx * d.z);
  const float cz = __builtin_fmaf(tx, d.y, -ty * d.x);
  const float u = __builtin_fmaf(T.e2[0], cx, __builtin_fmaf(T.e2[1], cy, T.e2[2] * cz));
  const float v = __builtin_fmaf(T.e1n[0], cx, __builtin_fmaf(T.e1n[1], cy, T.e1n[2] * cz));
  const float det = __builtin_fmaf(T.nn[0], d.x, __builtin_fmaf(T.nn[1], d.y, T.nn[2] * d.z));
  const float tt = __builtin_fmaf(T.nn[0], tx, __builtin_fmaf(T.nn[1], ty, T.nn[2] * tz));
  const float t = tt * rcp(-det);
  const float g = fminf(fminf(fminf(u, v), det - (u + v)), det - 0.000001f);
  const float ts = g >= 0.0f ? t : -1.0f;
  const bool acc = __float_as_uint(ts) < __float_as_uint(best);
  best = acc ? ts : best;
  tc = acc ? ts : tc;
}

// tri_test_t on a face's LTri record (shadow rays to a light with records)
template <class LR>
__device__ __forceinline__ void ltri_test_t(const LR& L, F3 o, float& best, float& tc) {
  const float ts = ltri_t(L, o);
  const bool acc = __float_as_uint(ts) < __float_as_uint(best);
  best = acc ? ts : best;
  tc = acc ? ts : tc;
}

// The faces listed at ent[b, e) against the rays of the batch's samples
// whose bit is set in fl (wave-uniform), each face record fetched once for
// all of them. Camera rays (KEY): list_search's (t, face) key. Shadow rays
// (!KEY): tri_test_t and the exact early exit (a sample's lane retires once
// it holds a hit with t <= stop; the search ends when no lane the list is
// for — own[k], the lanes whose ray lies in this cell — is left: the other
// lanes test these faces only as a harmless superset, their own cell is
// searched in its turn).
// diag (RTMI_DIAG_LANES builds, else nullptr): += the lanes still searching
// at each face test of each flagged sample (lane occupancy of the search).
// RTMI_LDS_STAGE (default 1; 0 for the A/B): each step's four face records
// staged through the wave's LDS slice instead of one scalar load per record
// (DESIGN.md "LDS staging": C3 0.912 -> 0.895 ms, C5 79.5 -> 78.4 ms).
#ifndef RTMI_LDS_STAGE
#define RTMI_LDS_STAGE 1
#endif
// Shadow searches (!KEY) test the light's LTri records at lb (lrec_of:
// every light with a grid has them), camera searches (KEY) the TriFast
// records of the tree. RTMI_GRID_REC (default 1): a shadow search reads the
// records in entry order instead, lb = the cell-ordered copy aligned with
// `ent` (grid_rec_of: entry k's record at lb + 64 k) — one load per step,
// not the entries and then the records they name; 0 for the A/B.
template <int S, bool KEY>
__device__ __forceinline__ int list_search_batch(KP p, const int32_t* ent, int b, int e, unsigned fl,
                                                  const F3 (&ro)[S], const F3 (&rd)[S], const float (&stop)[S],
                                                  const unsigned long long (&own)[S], unsigned long long (&key)[S],
                                                  float (&best)[S], float (&tc)[S], unsigned* diag = nullptr,
                                                  const char* lb = nullptr) {
  constexpr bool kCellRec = !KEY && RTMI_GRID_REC;
  // the record of entry k
  auto rec_at = [&](int k) -> const char* {
    return kCellRec ? lb + (size_t)(unsigned)k * sizeof(LTri) : lb + (unsigned)cp(ent)[k];
  };
  const int b_in = b;  // returns the number of faces tested (diagnostics)
  auto lanes = [&]() {
    if (diag) {
#pragma unroll
      for (int k = 0; k < S; ++k)
        if ((fl >> k) & 1u) *diag += pc(bal(tc[k] >= 0.0f));
    }
  };
  if constexpr (!KEY) {
    // a cell's first face alone: it is the one covering most of the cell
    // (rt_bins.cpp), so lanes in the umbra retire after one test
    if (b < e) {
      const LRegs T = load_ltri((const RT_CONST LTri*)rec_at(b));
      lanes();
      unsigned long long left = 0ull;
#pragma unroll
      for (int k = 0; k < S; ++k)
        if ((fl >> k) & 1u) {
          ltri_test_t(T, ro[k], best[k], tc[k]);
          tc[k] = tc[k] <= stop[k] ? -1.0f : tc[k];
          left |= bal(tc[k] >= 0.0f) & own[k];
        }
      if (left == 0ull) return 1;
      ++b;
    }
  }
  // LDS staging (RTMI_LDS_STAGE, DESIGN.md "LDS staging"): the 4 face
  // records of a step staged through the wave's LDS slice — lane 16 j + w
  // loads dword w of record j (one coalesced vector load for all four), then
  // every lane reads each record back as a broadcast (ds_read_b128 x 4) —
  // instead of one scalar load per record. 1: both searches, 2: the shadow
  // (cell list) searches only, 3: the camera (pixel list) searches only.
  constexpr bool kStage = RTMI_LDS_STAGE == 1 || (RTMI_LDS_STAGE == 2 && !KEY) || (RTMI_LDS_STAGE == 3 && KEY);
#if RTMI_LDS_STAGE
  __shared__ uint4 stage_lds[4][16];
  uint4* stage = stage_lds[threadIdx.x >> 6];
#else
  uint4* stage = nullptr;
#endif
  for (int k0 = b; k0 < e; k0 += 4) {
    int r[4] = {0, 0, 0, 0};
    if constexpr (!kCellRec) {
      const RT_CONST int32_t* q = cp(ent) + k0;
      r[0] = q[0], r[1] = q[1], r[2] = q[2], r[3] = q[3];
    }
    if constexpr (kStage) {
      const int lane = (int)__lane_id(), j = lane >> 4, w = lane & 15;
      if constexpr (kCellRec) {  // the step's four records are 256 contiguous bytes
        const unsigned int* src = (const unsigned int*)rec_at(k0);
        ((unsigned int*)stage)[lane] = k0 + j < e ? src[lane] : 0u;
      } else {
        const int rj = j == 0 ? r[0] : j == 1 ? r[1] : j == 2 ? r[2] : r[3];
        const unsigned int* src = (const unsigned int*)((KEY ? (const char*)p->tree : lb) + (unsigned)rj);
        ((unsigned int*)stage)[lane] = k0 + j < e ? src[w] : 0u;
      }
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j > 0 && k0 + j >= e) break;
      if constexpr (KEY) {
        TriRegs T;
        if constexpr (kStage) {
          const uint4 a = stage[4 * j + 0], bq = stage[4 * j + 1], c = stage[4 * j + 2], d4 = stage[4 * j + 3];
          T.v0[0] = __uint_as_float(a.x), T.v0[1] = __uint_as_float(a.y), T.v0[2] = __uint_as_float(a.z);
          T.id = a.w;
          T.e2[0] = __uint_as_float(bq.x), T.e2[1] = __uint_as_float(bq.y), T.e2[2] = __uint_as_float(bq.z);
          T.e1n[0] = __uint_as_float(c.x), T.e1n[1] = __uint_as_float(c.y), T.e1n[2] = __uint_as_float(c.z);
          T.nn[0] = __uint_as_float(d4.x), T.nn[1] = __uint_as_float(d4.y), T.nn[2] = __uint_as_float(d4.z);
        } else {
          (void)stage;
          T = load_tri(rec<TriFast>(p, r[j]));
        }
        lanes();
#pragma unroll
        for (int k = 0; k < S; ++k)
          if ((fl >> k) & 1u) tri_test(T, ro[k], rd[k], key[k], tc[k]);
      } else {
        LRegs T;
        if constexpr (kStage) {
          const uint4 a = stage[4 * j + 0], bq = stage[4 * j + 1], c = stage[4 * j + 2], d4 = stage[4 * j + 3];
          T.p[0] = __uint_as_float(a.x), T.p[1] = __uint_as_float(a.y), T.p[2] = __uint_as_float(a.z);
          T.cu = __uint_as_float(a.w);
          T.q[0] = __uint_as_float(bq.x), T.q[1] = __uint_as_float(bq.y), T.q[2] = __uint_as_float(bq.z);
          T.cv = __uint_as_float(bq.w);
          T.tv[0] = __uint_as_float(c.x), T.tv[1] = __uint_as_float(c.y), T.tv[2] = __uint_as_float(c.z);
          T.ct = __uint_as_float(c.w);
          T.id = d4.x;
        } else {
          (void)stage;
          T = load_ltri((const RT_CONST LTri*)(kCellRec ? rec_at(k0 + j) : lb + (unsigned)r[j]));
        }
        lanes();
#pragma unroll
        for (int k = 0; k < S; ++k)
          if ((fl >> k) & 1u) ltri_test_t(T, ro[k], best[k], tc[k]);
      }
    }
    if constexpr (!KEY) {
      unsigned long long left = 0ull;
#pragma unroll
      for (int k = 0; k < S; ++k)
        if ((fl >> k) & 1u) {
          tc[k] = tc[k] <= stop[k] ? -1.0f : tc[k];
          left |= bal(tc[k] >= 0.0f) & own[k];
        }
      if (left == 0ull) return min(e, k0 + 4) - b_in;
    }
  }
  return e - b_in;
}

// The mesh's AABB gate (TriangleMesh.intersect, geom.nim:339-341) in the
// traversal's slab form, as trace() forms it: a ray starting inside the box
// misses.
__device__ __forceinline__ bool mesh_gate(const FObj& ob, const SlabRay& sr) {
  const float ax = __builtin_fmaf(ob.lo[0], sr.ni.x, -sr.oi.x), bx = __builtin_fmaf(ob.hi[0], sr.ni.x, -sr.oi.x);
  const float ay = __builtin_fmaf(ob.lo[1], sr.ni.y, -sr.oi.y), by = __builtin_fmaf(ob.hi[1], sr.ni.y, -sr.oi.y);
  const float az = __builtin_fmaf(ob.lo[2], sr.ni.z, -sr.oi.z), bz = __builtin_fmaf(ob.hi[2], sr.ni.z, -sr.oi.z);
  const float gmin = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
  const float gmax = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz)) * 1.00000024f;
  return gmin <= gmax && gmin >= 0.0f;
}

// General pixels, S samples per lane at once (two-class launches: the
// pixels that are not lean). Scenes of one mesh object (FastParams
// .shadow_mesh), analytic objects and distant lights only, no reflection;
// one-pixel waves with the pixel's record (pinfo) and its camera-ray list.
// The same per-sample arithmetic as shade_path / trace / mesh_search —
// camera rays search the pixel's face list, shadow rays to a light whose
// skip bit is clear search their light-grid cells with the exact early
// exit — with each face record, object record and loop step paid once per
// 64 x S rays instead of per 64. No BVH here: when a shadow ray would need
// it (a light without a grid, an origin beyond the grid's float32-safe
// radius) the batch returns false
// before adding anything and the caller renders the whole pixel with the
// one-sample loop. Stats go to `wi` (committed by the caller). Frames and
// Stats bit-identical to the one-sample loop (test_gpu_split.py against
// RT_FLAG_NO_BATCH / NO_SPLIT / NO_BINNING).
template <unsigned F, int S>
__device__ __forceinline__ bool gen_batch(KP p, const GroupPix& gp, int it0, const LdsF* tb, unsigned pinfo,
                                          LdsF* ls, Acc& acc, Stats32& wi) {
  static_assert(3 * S <= kLdsSlots, "albedo stash: 3 LDS slots per sample");
  // kernel arguments re-read through a laundered pointer at each stage
  // (params()): hoisted, the many fields this path reads stay pinned in
  // SGPRs across the whole batch and spill
  p = params();
  const F3 o = f3(p->cam[0], p->cam[1], p->cam[2]);
  F3 d[S];
  bool sv[S];
  batch_dirs<F, S>(p, gp, it0, tb, d, sv);
  unsigned nprim = 0u;
  // th: -1 invalid sample, +inf sky, else the closest hit's t (lean_batch)
  float th[S];
  int hob[S], htri[S];
#pragma unroll
  for (int k = 0; k < S; ++k) {
    nprim += pc(bal(sv[k]));
    th[k] = sv[k] ? finf() : -1.0f;
    hob[k] = -1;
    htri[k] = -1;
  }
  const int nobj = p->nobj, mesh = p->shadow_mesh;
  unsigned hitl = 0u;
  // camera rays: trace (renderer.nim:47-67) over the objects in scene order
  for (int i = 0; i < nobj; ++i) {
    p = params();
    const FObj ob = at(p->objs, i);
    if (i == mesh) {
      // an empty pixel list: no camera ray of the pixel can hit the mesh
      // (trace's no_mesh: the gate's verdict cannot matter)
      if ((pinfo & kPixCount) == 0u || ob.root < 0) continue;
#ifdef RTMI_DIAG_GEN_NOCAM
      continue;  // diagnostic build only (wrong images): the camera searches' share
#endif
      F3 ro[S], rd[S];
      unsigned long long key[S], key0[S];
      float tc[S], unused[S];
      unsigned long long anyp = 0ull, nomask[S];
#pragma unroll
      for (int k = 0; k < S; ++k) {
        to_object<F>(p, ob, i, o, d[k], ro[k], rd[k]);
        const bool part = sv[k] && mesh_gate(ob, slab_ray(ro[k], rd[k]));
        tc[k] = part ? th[k] : -1.0f;
        key0[k] = part ? tkey(th[k], 0u) : 0ull;
        key[k] = key0[k];
        unused[k] = 0.0f;
        nomask[k] = 0ull;
        anyp |= bal(part);
      }
      if (anyp != 0ull) {  // the wave's one pixel: one list for every sample (gen_batch's caller
                           // sends a pixel whose list overflowed its slots to the one-sample loop)
        const int pu = __builtin_amdgcn_readfirstlane(gp.y * p->width + gp.x);
        const int b = pu << p->slot_lg;
        list_search_batch<S, true>(p, p->pix_slots, b, b + (int)(pinfo & kPixCount), (1u << S) - 1u,
                                   ro, rd, unused, nomask, key, unused, tc);
      }
#pragma unroll
      for (int k = 0; k < S; ++k) {  // found => 0 <= t < th: the hit counts (trace's update rule)
        const bool c = key[k] != key0[k];
        th[k] = c ? __uint_as_float((unsigned int)(key[k] >> 32)) : th[k];
        hob[k] = c ? i : hob[k];
        htri[k] = c ? (int)(unsigned int)key[k] : htri[k];
        hitl += c ? 1u : 0u;
      }
      continue;
    }
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const float t = analytic_t<F>(p, ob, i, o, d[k]);
      const bool c = t >= 0.0f && t < th[k];  // (t >= 0 ? t : inf) < th, th <= inf
      th[k] = c ? t : th[k];
      hob[k] = c ? i : hob[k];
      hitl += c ? 1u : 0u;
    }
  }
  // shade (renderer.nim:71-127): normals per distinct object hit (mesh:
  // the face normal by face id, renderer.nim:84-88), shadow origins
  unsigned long long litm[S], pend[S], skym[S];  // lit / sky lanes per sample
  F3 N[S], so[S];
#pragma unroll
  for (int k = 0; k < S; ++k) {
    litm[k] = m_lt(th[k], finf()) & m_ge(th[k], 0.0f);
    skym[k] = bal(th[k] == finf());
    pend[k] = litm[k];
    N[k] = f3(0.0f, 0.0f, 0.0f);
    so[k] = f3(__builtin_fmaf(d[k].x, th[k], o.x), __builtin_fmaf(d[k].y, th[k], o.y),
               __builtin_fmaf(d[k].z, th[k], o.z));  // the hit point until N is known
  }
  for (;;) {
    const int oi = first_pending<S>(pend, hob);
    if (oi < 0) break;
    int oi_cmp = oi;
    asm volatile("" : "+s"(oi_cmp));
    p = params();
    const FObj ob = at(p->objs, oi);
    const RT_CONST FObjX& ox = at(p->objx, oi);
    const bool is_mesh = (F & F_MESH) && ob.type == GEOM_MESH;
    const int nbase = ox.normal_base;
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const unsigned long long mine = bal(hob[k] == oi_cmp) & pend[k];
      pend[k] &= ~mine;
      const bool mi = lane_in(mine);
      F3 n;
      if (is_mesh) {
        // every lane loads (face 0 for the others): no exec-mask branch
        const float* fn = p->normals + 3 * (size_t)(nbase + (mi ? htri[k] : 0));
        n = f3(fn[0], fn[1], fn[2]);
      } else {
        F3 ho, unused;
        to_object<F>(p, ob, oi, so[k], f3(0.0f, 0.0f, 0.0f), ho, unused);
        n = analytic_normal<F>(ob, ho);
      }
      if ((F & F_XF_GENERAL) && ob.xf == XF_GENERAL) {  // object_to_world * n, not re-normalised
        const float* m = ox.o2w;
        n = f3(__builtin_fmaf(m[0], n.x, __builtin_fmaf(m[3], n.y, m[6] * n.z)),
               __builtin_fmaf(m[1], n.x, __builtin_fmaf(m[4], n.y, m[7] * n.z)),
               __builtin_fmaf(m[2], n.x, __builtin_fmaf(m[5], n.y, m[8] * n.z)));
      }
      N[k] = f3(mi ? n.x : N[k].x, mi ? n.y : N[k].y, mi ? n.z : N[k].z);
      // albedo / pi waits in LDS (slots 3k..3k+2) until the lights are summed
      if (mi) lds_put3(ls, 3 * k, f3(ox.albedo_pi[0], ox.albedo_pi[1], ox.albedo_pi[2]));
    }
  }
  const float bias = p->bias;
#pragma unroll
  for (int k = 0; k < S; ++k)
    so[k] = f3(__builtin_fmaf(N[k].x, bias, so[k].x), __builtin_fmaf(N[k].y, bias, so[k].y),
               __builtin_fmaf(N[k].z, bias, so[k].z));
  // one shadow ray per distant light and lit sample
  F3 E[S];
  unsigned long long anylit = 0ull;
  unsigned nlit = 0u;
#pragma unroll
  for (int k = 0; k < S; ++k) {
    E[k] = f3(0.0f, 0.0f, 0.0f);
    anylit |= litm[k];
    nlit += pc(litm[k]);
  }
  const int nl = anylit ? p->nlight : 0;
  const unsigned skipw = pinfo >> 24;  // bit l: no shadow ray to light l can meet the mesh
  for (int li = 0; li < nl; ++li) {
    p = params();
    const FLight L = at(p->lights, li);
    const F3 sd = f3(-L.v[0], -L.v[1], -L.v[2]);
    float ts[S];  // unlit samples start at 0 (take no part)
#pragma unroll
    for (int k = 0; k < S; ++k) ts[k] = lane_in(litm[k]) ? finf() : 0.0f;
    for (int i = 0; i < nobj; ++i) {
      p = params();
      const FObj ob = at(p->objs, i);
      if (i == mesh) {
        if ((li < 8 && ((skipw >> li) & 1u) != 0u) || ob.root < 0) continue;
#ifdef RTMI_DIAG_GEN_NOSHADOW
        continue;  // diagnostic build only (wrong images): the shadow searches' share
#endif
        F3 ro[S], rd[S];
        unsigned long long pm[S], anyp = 0ull;
#pragma unroll
        for (int k = 0; k < S; ++k) {
          to_object<F>(p, ob, i, so[k], sd, ro[k], rd[k]);
          pm[k] = bal(lane_in(litm[k]) && mesh_gate(ob, slab_ray(ro[k], rd[k])));
          anyp |= pm[k];
        }
        if (anyp == 0ull) continue;  // no lane enters the mesh's box
#ifdef RTMI_DIAG_GEN_NOSHADOWSEARCH
        continue;  // diagnostic build only (wrong images): the gated shadow searches' share
#endif
        if (!p->grids || p->grids[li].gu <= 0) return false;  // the BVH: the caller's one-sample loop
        // mesh_search: the exact early exit's stop distance (the analytic
        // objects after the mesh), clamped below each lane's initial limit
        float stop[S], tc[S], best[S];
        unsigned long long unused[S];
#pragma unroll
        for (int k = 0; k < S; ++k) stop[k] = finf();
        for (int j = i + 1; j < nobj; ++j) {
          const FObj oj = at(p->objs, j);
#pragma unroll
          for (int k = 0; k < S; ++k) {
            const float tj = analytic_t<F>(p, oj, j, so[k], sd);
            stop[k] = tj >= 0.0f ? fminf(stop[k], tj) : stop[k];
          }
        }
        // the light grid's cells (rt_bins.h); a float32-safe lane off the
        // grid can hit no face
        const RT_CONST LightGrid& G = cp(p->grids)[li];
        int cell[S];
        unsigned long long todo[S], left = 0ull, unsafe = 0ull;
#pragma unroll
        for (int k = 0; k < S; ++k) {
          const bool part = lane_in(pm[k]);
          stop[k] = fminf(stop[k], __uint_as_float(__float_as_uint(ts[k]) - 1u));
          tc[k] = part ? ts[k] : -1.0f;
          best[k] = part ? ts[k] : 0.0f;
          unused[k] = 0ull;
          const F3 r = ro[k];
          const float gu = __builtin_fmaf(r.x, G.e1[0], __builtin_fmaf(r.y, G.e1[1], r.z * G.e1[2]));
          const float gv = __builtin_fmaf(r.x, G.e2[0], __builtin_fmaf(r.y, G.e2[1], r.z * G.e2[2]));
          const float fu = (gu - G.u0) * G.inv_h, fv = (gv - G.v0) * G.inv_h;
          const bool safe = fmaxf(fmaxf(fabsf(r.x), fabsf(r.y)), fabsf(r.z)) <= G.rmax;
          const bool on = fu >= 0.0f && fu < (float)G.gu && fv >= 0.0f && fv < (float)G.gv;
          cell[k] = safe && on ? G.off_base + (int)fv * G.gu + (int)fu : -1;
          todo[k] = bal(part && cell[k] >= 0);
          unsafe |= bal(part && !safe);
          left |= todo[k];
        }
        if (unsafe != 0ull) return false;
        const int32_t* bent = p->grid_ent + G.ent_base;
        // every distinct cell of the batch's shadow rays in turn (each round
        // retires at least the lane the cell was taken from)
#ifdef RTMI_DIAG_GEN_COUNT
        wi.v[STAT_LANE_NODES] += 1u;  // diagnostic: searched (light, batch) visits
#endif
        while (left != 0ull) {
          int kb = -1;
#pragma unroll
          for (int k = S - 1; k >= 0; --k)
            if (todo[k]) kb = __builtin_amdgcn_readlane(cell[k], (int)__builtin_ctzll(todo[k]));
          unsigned fl = 0u;
          unsigned long long own[S];
          left = 0ull;
#pragma unroll
          for (int k = 0; k < S; ++k) {
            own[k] = bal(cell[k] == kb) & todo[k];
            fl |= own[k] != 0ull ? (1u << k) : 0u;
            todo[k] &= ~own[k];
            left |= todo[k];
          }
#ifdef RTMI_DIAG_GEN_COUNT
          wi.v[STAT_NODE_FETCH] += 1u;  // diagnostic: cells searched
          wi.v[STAT_TRI_FETCH] += (unsigned)(cp(p->grid_off)[kb + 1] - cp(p->grid_off)[kb]) * (unsigned)__builtin_popcount(fl);
#endif
          list_search_batch<S, false>(p, bent, cp(p->grid_off)[kb], cp(p->grid_off)[kb + 1], fl, ro, rd, stop,
                                      own, unused, best, tc, nullptr, grid_rec_of(p, li, G));
        }
#pragma unroll
        for (int k = 0; k < S; ++k) {  // found => 0 <= t < ts: the hit counts
          const bool c = lane_in(pm[k]) && __float_as_uint(best[k]) != __float_as_uint(ts[k]);
          ts[k] = c ? best[k] : ts[k];
          hitl += c ? 1u : 0u;
        }
        continue;
      }
#pragma unroll
      for (int k = 0; k < S; ++k) {
        const float t = analytic_t<F>(p, ob, i, so[k], sd);
        const bool c = t >= 0.0f && t < ts[k];
        ts[k] = c ? t : ts[k];
        hitl += c ? 1u : 0u;
      }
    }
#pragma unroll
    for (int k = 0; k < S; ++k) {  // unoccluded: shadeDiffuse (shader.nim:12-17)
      const bool vis = lane_in(litm[k]) && !(ts[k] < finf());
      irr_add(E[k], L.ci, vis ? fmaxf(dot3(N[k], sd), 0.0f) : 0.0f);
    }
  }
  // the samples' colours in order: albedo / pi x E, the background for the sky
  p = params();
  const F3 bg = f3(p->bg[0], p->bg[1], p->bg[2]);
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const bool lt = lane_in(litm[k]), sky = lane_in(skym[k]);
    const F3 a = mul3(lds_get3(ls, 3 * k), E[k]);
    const F3 c = f3(lt ? a.x : (sky ? bg.x : 0.0f), lt ? a.y : (sky ? bg.y : 0.0f),
                    lt ? a.z : (sky ? bg.z : 0.0f));
    acc_add3(acc, c.x, c.y, c.z);
  }
  wi.v[STAT_PRIMARY] += nprim;
  wi.v[STAT_SHADOW] += (unsigned)nl * nlit;
#ifdef RTMI_DIAG_GEN_COUNT
  wi.v[STAT_LANE_TRIS] += 1u;  // diagnostic: batches
#endif
  wi.v[STAT_HITS] += wave_sum(hitl);
  return true;
}

// General pixels of the one-plane scenes (k_render_lean1's: one mesh + one
// translated plane, distant lights, akGrid m | 64, every sample valid):
// gen_batch with the two objects written out in scene order instead of the
// object / dispatch loops — the plane's camera and shadow tests in
// k_render_lean1's form, its normal (0, 1, 0), the albedo a select of the
// two objects' (no LDS stash), the camera's cx terms per lane and pixel.
// The mesh searches (pixel list, light-grid cells, the early exit's stop)
// are gen_batch's, unchanged. Returns false, before adding anything, where
// gen_batch does (a shadow ray that needs the BVH). Frames and Stats
// bit-identical to gen_batch (tests/test_gpu_split.py, RT_FLAG_NO_GEN1).
// RTMI_GEN1_COMPACT=1 (A/B, row n2): the two samples' rays of a light cell
// packed into one slot when they fit one wave (gen1_batch's cell loop).
// Exact (frames and Stats bit-identical, GPU parity tests green) but slower:
// C3 0.901 -> 0.918 ms, C5 78.5 -> 79.4 ms — the pairing and permutes cost
// more than the face tests they save, and the kernel's spills grow from 4
// to 18 VGPRs (DESIGN.md "Live-ray compaction of the light-cell searches").
#ifndef RTMI_GEN1_COMPACT
#define RTMI_GEN1_COMPACT 0
#endif
template <int S, int NL>
__device__ __forceinline__ bool gen1_batch(KP p, const GroupPix& gp, int pu, int it0, unsigned pinfo, Acc& acc,
                                           Stats32& wi) {
  p = params();
  const int mesh = p->shadow_mesh, po = 1 - mesh;  // the scene's two objects
  const F3 o = f3(p->cam[0], p->cam[1], p->cam[2]);
  F3 d[S];
  {
    const int mm = p->grid_m - 1, lg = p->log2_grid_m;
    const float st = p->sample_step, of = p->sample_off;
    const float px = (float)gp.x + __builtin_fmaf((float)(gp.sub & mm), st, of);
    const float cx = (px - p->cam_b) * p->cam_a;
    const float q0 = __builtin_fmaf(cx, cx, 1.0f);
    const float ax = __builtin_fmaf(cx, p->cam[3], -p->cam[9]), ay = __builtin_fmaf(cx, p->cam[4], -p->cam[10]),
                az = __builtin_fmaf(cx, p->cam[5], -p->cam[11]);
#pragma unroll
    for (int k = 0; k < S; ++k) {  // camera_ray_dir, the cx terms formed once
      const int s = (it0 + k) * 64 + gp.sub;
      const float py = (float)gp.y + __builtin_fmaf((float)(s >> lg), st, of);
      const float cy = (p->cam_d - py) * p->cam_c;
      const float rl = rsq(__builtin_fmaf(cy, cy, q0));
      d[k] = f3(__builtin_fmaf(cy, p->cam[6], ax) * rl, __builtin_fmaf(cy, p->cam[7], ay) * rl,
                __builtin_fmaf(cy, p->cam[8], az) * rl);
    }
  }
  float th[S];
  bool hm[S];  // the closest hit is the mesh's
  int htri[S];
#pragma unroll
  for (int k = 0; k < S; ++k) {
    th[k] = finf();
    hm[k] = false;
    htri[k] = -1;
  }
  unsigned hitl = 0u;
  const FObj mob = at(p->objs, mesh);
  const float pty = at(p->objs, po).t[1];
  // trace (renderer.nim:47-67) of the camera rays: the two objects in order
  auto camera_plane = [&]() {
    const float nroy = -(o.y + pty);
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const float t = fabsf(d[k].y) > 1e-6f ? nroy * rcp(d[k].y) : -finf();
      const bool c = t >= 0.0f && t < th[k];
      th[k] = c ? t : th[k];
      hm[k] = c ? false : hm[k];
      hitl += c ? 1u : 0u;
    }
  };
  auto camera_mesh = [&]() {
    if ((pinfo & kPixCount) == 0u || mob.root < 0) return;  // an empty pixel list: no camera ray can hit it
#ifdef RTMI_DIAG_GEN_NOCAM
    return;  // diagnostic build only (wrong images): the camera searches' share
#endif
    F3 ro[S], rd[S];
    unsigned long long key[S], key0[S], anyp = 0ull, nomask[S];
    float tc[S], unused[S];
#pragma unroll
    for (int k = 0; k < S; ++k) {
      ro[k] = f3(o.x + mob.t[0], o.y + mob.t[1], o.z + mob.t[2]);
      rd[k] = d[k];
      const bool part = mesh_gate(mob, slab_ray(ro[k], rd[k]));
      tc[k] = part ? th[k] : -1.0f;
      key0[k] = part ? tkey(th[k], 0u) : 0ull;
      key[k] = key0[k];
      unused[k] = 0.0f;
      nomask[k] = 0ull;
      anyp |= bal(part);
    }
    if (anyp != 0ull) {
      const KP q = params();
      const int b = pu << q->slot_lg;
#ifdef RTMI_DIAG_LANES  // diagnostic: camera face tests (x samples) and the lanes still searching
      unsigned dl = 0u;
      wi.v[STAT_TRI_FETCH] += (unsigned)(pinfo & kPixCount) * (unsigned)S;
      list_search_batch<S, true>(q, q->pix_slots, b, b + (int)(pinfo & kPixCount), (1u << S) - 1u,
                                 ro, rd, unused, nomask, key, unused, tc, &dl);
      wi.v[STAT_LANE_TRIS] += dl;
#else
      list_search_batch<S, true>(q, q->pix_slots, b, b + (int)(pinfo & kPixCount), (1u << S) - 1u,
                                 ro, rd, unused, nomask, key, unused, tc);
#endif
    }
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const bool c = key[k] != key0[k];
      th[k] = c ? __uint_as_float((unsigned int)(key[k] >> 32)) : th[k];
      hm[k] = c ? true : hm[k];
      htri[k] = c ? (int)(unsigned int)key[k] : htri[k];
      hitl += c ? 1u : 0u;
    }
  };
  if (mesh == 0) {
    camera_mesh();
    camera_plane();
  } else {
    camera_plane();
    camera_mesh();
  }
  // shade (renderer.nim:71-127): N = the face normal (renderer.nim:84-88) or
  // the plane's (0, 1, 0); the shadow origins hitW + N * bias
  p = params();
  unsigned long long litm[S], anylit = 0ull, anymesh = 0ull;
  unsigned nlit = 0u;
  F3 N[S], so[S];
#pragma unroll
  for (int k = 0; k < S; ++k) {
    litm[k] = m_lt(th[k], finf()) & m_ge(th[k], 0.0f);
    anylit |= litm[k];
    nlit += pc(litm[k]);
    anymesh |= bal(hm[k]) & litm[k];
    so[k] = f3(__builtin_fmaf(d[k].x, th[k], o.x), __builtin_fmaf(d[k].y, th[k], o.y),
               __builtin_fmaf(d[k].z, th[k], o.z));
  }
  const int nbase = at(p->objx, mesh).normal_base;
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const bool lt = lane_in(litm[k]);
    F3 n = f3(0.0f, 1.0f, 0.0f);
    if (anymesh != 0ull) {  // every lane loads (face 0 for the others): no exec-mask branch
      const bool mi = lt && hm[k];
      const float* fn = p->normals + 3 * (size_t)(nbase + (mi ? htri[k] : 0));
      n = f3(mi ? fn[0] : n.x, mi ? fn[1] : n.y, mi ? fn[2] : n.z);
    }
    N[k] = f3(lt ? n.x : 0.0f, lt ? n.y : 0.0f, lt ? n.z : 0.0f);
  }
  const float bias = p->bias;
#pragma unroll
  for (int k = 0; k < S; ++k)
    so[k] = f3(__builtin_fmaf(N[k].x, bias, so[k].x), __builtin_fmaf(N[k].y, bias, so[k].y),
               __builtin_fmaf(N[k].z, bias, so[k].z));
  // one shadow ray per distant light and lit sample
  F3 E[S];
#pragma unroll
  for (int k = 0; k < S; ++k) E[k] = f3(0.0f, 0.0f, 0.0f);
  const unsigned skipw = pinfo >> 24;
  if (anylit != 0ull) {
#pragma unroll
    for (int li = 0; li < NL; ++li) {
      p = params();
      const FLight L = at(p->lights, li);
      const F3 sd = f3(-L.v[0], -L.v[1], -L.v[2]);
      // the plane's shadow test (lean1's form: NaN multiplier when parallel)
      const float mulp = fabsf(sd.y) > 1e-6f ? rcp(sd.y) : __builtin_nanf("");
      float ts[S], tpl[S];
#pragma unroll
      for (int k = 0; k < S; ++k) {
        ts[k] = lane_in(litm[k]) ? finf() : 0.0f;
        tpl[k] = -(so[k].y + pty) * mulp;
      }
      auto shadow_plane = [&]() {
#pragma unroll
        for (int k = 0; k < S; ++k) {
          const bool c = tpl[k] >= 0.0f && tpl[k] < ts[k];
          ts[k] = c ? tpl[k] : ts[k];
          hitl += c ? 1u : 0u;
        }
      };
      // the mesh (gen_batch's search), false: the BVH would be needed
      auto shadow_mesh = [&]() -> bool {
        if (((skipw >> li) & 1u) != 0u || mob.root < 0) return true;
#ifdef RTMI_DIAG_GEN_NOSHADOW
        return true;
#endif
        F3 ro[S], rd[S];
        unsigned long long pm[S], anyp = 0ull;
#pragma unroll
        for (int k = 0; k < S; ++k) {
          ro[k] = f3(so[k].x + mob.t[0], so[k].y + mob.t[1], so[k].z + mob.t[2]);
          rd[k] = sd;
          pm[k] = bal(lane_in(litm[k]) && mesh_gate(mob, slab_ray(ro[k], rd[k])));
#ifdef RTMI_DIAG_GEN_NOMESHORIGIN
          pm[k] &= ~bal(hm[k]);  // diagnostic build only (wrong images): mesh-origin shadow rays skip the mesh
#endif
          anyp |= pm[k];
        }
        if (anyp == 0ull) return true;
#ifdef RTMI_DIAG_GEN_NOSHADOWSEARCH
        return true;  // diagnostic build only (wrong images): the gated shadow searches' share
#endif
        const KP q = params();
        if (!q->grids || q->grids[li].gu <= 0) return false;
        // the exact early exit's stop: the plane after the mesh (if it is)
        float stop[S], tc[S], best[S];
        unsigned long long unused[S];
#pragma unroll
        for (int k = 0; k < S; ++k) {
          stop[k] = finf();
          if (mesh == 0) stop[k] = tpl[k] >= 0.0f ? fminf(stop[k], tpl[k]) : stop[k];
        }
        const RT_CONST LightGrid& G = cp(q->grids)[li];
#if RTMI_GEN1_COMPACT
        __shared__ int cmp_lds_all[4][64];  // per wave: the lane pairing of a compacted cell search
        int* cmp_lds = cmp_lds_all[threadIdx.x >> 6];
#endif
        int cell[S];
        unsigned long long todo[S], left = 0ull, unsafe = 0ull;
#pragma unroll
        for (int k = 0; k < S; ++k) {
          const bool part = lane_in(pm[k]);
          stop[k] = fminf(stop[k], __uint_as_float(__float_as_uint(ts[k]) - 1u));
          tc[k] = part ? ts[k] : -1.0f;
          best[k] = part ? ts[k] : 0.0f;
          unused[k] = 0ull;
          const F3 r = ro[k];
          const float gu = __builtin_fmaf(r.x, G.e1[0], __builtin_fmaf(r.y, G.e1[1], r.z * G.e1[2]));
          const float gv = __builtin_fmaf(r.x, G.e2[0], __builtin_fmaf(r.y, G.e2[1], r.z * G.e2[2]));
          const float fu = (gu - G.u0) * G.inv_h, fv = (gv - G.v0) * G.inv_h;
          const bool safe = fmaxf(fmaxf(fabsf(r.x), fabsf(r.y)), fabsf(r.z)) <= G.rmax;
          const bool on = fu >= 0.0f && fu < (float)G.gu && fv >= 0.0f && fv < (float)G.gv;
          cell[k] = safe && on ? G.off_base + (int)fv * G.gu + (int)fu : -1;
          todo[k] = bal(part && cell[k] >= 0);
          unsafe |= bal(part && !safe);
          left |= todo[k];
        }
        if (unsafe != 0ull) return false;
        const int32_t* bent = q->grid_ent + G.ent_base;
        while (left != 0ull) {
          int kb = -1;
#pragma unroll
          for (int k = S - 1; k >= 0; --k)
            if (todo[k]) kb = __builtin_amdgcn_readlane(cell[k], (int)__builtin_ctzll(todo[k]));
          unsigned fl = 0u;
          unsigned long long own[S];
          left = 0ull;
#pragma unroll
          for (int k = 0; k < S; ++k) {
            own[k] = bal(cell[k] == kb) & todo[k];
            todo[k] &= ~own[k];
            left |= todo[k];
            fl |= own[k] != 0ull ? (1u << k) : 0u;
#ifdef RTMI_DIAG_GEN_COUNT
            wi.v[STAT_LANE_NODES] += pc(own[k]);  // diagnostic: rays in searched cells
#endif
          }
#ifdef RTMI_DIAG_GEN_NOTESTS
          continue;  // diagnostic build only (wrong images): the cell loop without its face tests
#endif
#if RTMI_GEN1_COMPACT
          // Both samples have rays in this cell and together they fit one
          // wave: sample 1's rays move into the lanes sample 0 leaves free
          // (ballot + v_mbcnt ranks, the lane pairing through LDS, the ray
          // state by ds_bpermute) and the cell's faces are tested once
          // instead of twice; each ray's tests and its retirement are
          // unchanged, so `best` (the only state the shade reads back: found /
          // not found, and its order against `stop`) is the two-slot
          // search's. Lanes outside the cell test faces as a harmless
          // superset either way (list_search_batch).
          if constexpr (S == 2) {
            const unsigned long long m0 = own[0], m1 = own[1], fr0 = ~own[0];
            const unsigned n1 = pc(m1);
            if (fl == 3u && pc(m0) + n1 <= 64u) {
              const int lane = (int)__lane_id();
              const unsigned r1 = __builtin_amdgcn_mbcnt_hi((unsigned)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m1, 0u));
              const unsigned rf = __builtin_amdgcn_mbcnt_hi((unsigned)(fr0 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)fr0, 0u));
              const bool src = lane_in(m1), dst = lane_in(fr0) && rf < n1;
              int* pair = cmp_lds;
              if (src) pair[r1] = lane;          // the r-th ray of sample 1 ...
              __builtin_amdgcn_wave_barrier();
              const int from = dst ? pair[rf] : lane;  // ... goes to the r-th free lane
              __builtin_amdgcn_wave_barrier();
              if (dst) pair[rf] = lane;
              __builtin_amdgcn_wave_barrier();
              const int to = src ? pair[r1] : lane;
              __builtin_amdgcn_wave_barrier();
              auto take = [&](float v0, float v1) {  // slot 0's value, or sample 1's from `from`
                const float m = __int_as_float(__builtin_amdgcn_ds_bpermute(from << 2, __float_as_int(v1)));
                return dst ? m : v0;
              };
              F3 ro_c[1] = {f3(take(ro[0].x, ro[1].x), take(ro[0].y, ro[1].y), take(ro[0].z, ro[1].z))};
              const F3 rd_c[1] = {rd[0]};  // (both samples: the light's direction)
              const float stop_c[1] = {take(stop[0], stop[1])};
              float best_c[1] = {take(best[0], best[1])}, tc_c[1] = {take(tc[0], tc[1])};
              const unsigned long long own_c[1] = {m0 | bal(dst)};
              unsigned long long key_c[1] = {0ull};
#ifdef RTMI_DIAG_LANES
              unsigned dl = 0u;
              const int nt = list_search_batch<1, false>(q, bent, cp(q->grid_off)[kb], cp(q->grid_off)[kb + 1], 1u, ro_c,
                                                         rd_c, stop_c, own_c, key_c, best_c, tc_c, &dl, grid_rec_of(q, li, G));
              wi.v[STAT_NODE_FETCH] += (unsigned)nt;
              wi.v[STAT_LANE_NODES] += dl;
#else
              (void)list_search_batch<1, false>(q, bent, cp(q->grid_off)[kb], cp(q->grid_off)[kb + 1], 1u, ro_c, rd_c,
                                                stop_c, own_c, key_c, best_c, tc_c, nullptr, grid_rec_of(q, li, G));
#endif
              // back: slot 0 in place, sample 1's rays from the lane they moved to
              const float b1 = __int_as_float(__builtin_amdgcn_ds_bpermute(to << 2, __float_as_int(best_c[0])));
              const float t1 = __int_as_float(__builtin_amdgcn_ds_bpermute(to << 2, __float_as_int(tc_c[0])));
              const bool in0 = lane_in(m0);
              best[0] = in0 ? best_c[0] : best[0];
              tc[0] = in0 ? tc_c[0] : tc[0];
              best[1] = src ? b1 : best[1];
              tc[1] = src ? t1 : tc[1];
              continue;
            }
          }
#endif
#ifdef RTMI_DIAG_LANES  // diagnostic: shadow face tests (x flagged samples) and the lanes still searching
          unsigned dl = 0u;
          const int nt = list_search_batch<S, false>(q, bent, cp(q->grid_off)[kb], cp(q->grid_off)[kb + 1], fl, ro, rd,
                                                     stop, own, unused, best, tc, &dl, grid_rec_of(q, li, G));
          wi.v[STAT_NODE_FETCH] += (unsigned)nt * (unsigned)__builtin_popcount(fl);
          wi.v[STAT_LANE_NODES] += dl;
#else
          const int nt = list_search_batch<S, false>(q, bent, cp(q->grid_off)[kb], cp(q->grid_off)[kb + 1], fl, ro, rd,
                                                     stop, own, unused, best, tc, nullptr, grid_rec_of(q, li, G));
#endif
#ifdef RTMI_DIAG_GEN_COUNT
          wi.v[STAT_NODE_FETCH] += 1u;                                      // diagnostic: cells searched
          wi.v[STAT_TRI_FETCH] += (unsigned)nt * (unsigned)__builtin_popcount(fl);  // wave face tests
#else
          (void)nt;
#endif
        }
#pragma unroll
        for (int k = 0; k < S; ++k) {  // found => 0 <= t < ts: the hit counts
          const bool c = lane_in(pm[k]) && __float_as_uint(best[k]) != __float_as_uint(ts[k]);
          ts[k] = c ? best[k] : ts[k];
          hitl += c ? 1u : 0u;
        }
        return true;
      };
      if (mesh == 0) {
        if (!shadow_mesh()) return false;
        shadow_plane();
      } else {
        shadow_plane();
        if (!shadow_mesh()) return false;
      }
#pragma unroll
      for (int k = 0; k < S; ++k) {  // unoccluded: shadeDiffuse (shader.nim:12-17)
        const bool vis = lane_in(litm[k]) && !(ts[k] < finf());
        irr_add(E[k], L.ci, vis ? fmaxf(dot3(N[k], sd), 0.0f) : 0.0f);
      }
    }
  }
  // the samples' colours in order: albedo / pi x E (the hit object's), the
  // background for the sky (every sample valid: not lit = sky)
  p = params();
  const RT_CONST FObjX& mx = at(p->objx, mesh);
  const RT_CONST FObjX& px_ = at(p->objx, po);
  const F3 am = f3(mx.albedo_pi[0], mx.albedo_pi[1], mx.albedo_pi[2]);
  const F3 ap = f3(px_.albedo_pi[0], px_.albedo_pi[1], px_.albedo_pi[2]);
  const F3 bg = f3(p->bg[0], p->bg[1], p->bg[2]);
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const bool lt = lane_in(litm[k]);
    const F3 alb = f3(hm[k] ? am.x : ap.x, hm[k] ? am.y : ap.y, hm[k] ? am.z : ap.z);
    const F3 a = mul3(alb, E[k]);
    acc_add3(acc, lt ? a.x : bg.x, lt ? a.y : bg.y, lt ? a.z : bg.z);
  }
  wi.v[STAT_PRIMARY] += (unsigned)(64 * S);
  wi.v[STAT_SHADOW] += (unsigned)NL * nlit;
  wi.v[STAT_HITS] += wave_sum(hitl);
  return true;
}

// multiJittered / correlatedMultiJittered (sampling.nim:39-113): the wave
// builds each of its pixels' (m, m) tables in LDS — canonical entries spread
// over the pixel's lanes, then the x shuffle with one lane per column and
// the y shuffle with one lane per row (each lane only touches its own column
// / row, so the sequential reference order holds per lane; rt_sampling.h
// draw indices). nullptr for the other samplers.
template <unsigned F>
__device__ __forceinline__ LdsF* sample_table(KP p, const GroupPix& gp, float* sample_lds, int wib, int L) {
  LdsF* tb = nullptr;
  if ((F & F_STOCHASTIC) && p->aa_kind >= 3) {
    const int m = p->grid_m, spp = p->spp;
    const uint64_t key = rng_pixel_key(p->seed, gp.x, gp.y);
    tb = (LdsF*)sample_lds + ((size_t)(wib * (64 / L) + (lane_id_fresh() >> p->log2_lanes)) * 2 * spp);
    volatile LdsF* t = tb;
    for (int e = gp.sub; e < spp; e += L) {
      double a, b;
      canonical_entry(key, m, e, a, b);
      t[e] = (float)a;
      t[spp + e] = (float)b;
    }
    const uint64_t bx = 2 * (uint64_t)spp;
    const uint64_t by = bx + (p->aa_kind == 3 ? (uint64_t)spp : (uint64_t)m);
    if (gp.sub < m) {
      const int i = gp.sub;  // column i: the x shuffle
      for (int j = 0; j < m; ++j) {
        const int k = rng_pick(rng_draw(key, p->aa_kind == 3 ? bx + (uint64_t)j * m + i : bx + (uint64_t)j), j, m);
        const float a = t[j * m + i], b = t[k * m + i];
        t[j * m + i] = b;
        t[k * m + i] = a;
      }
      const int j = gp.sub;  // row j: the y shuffle
      for (int ii = 0; ii < m; ++ii) {
        const int k = rng_pick(rng_draw(key, p->aa_kind == 3 ? by + (uint64_t)ii * m + j : by + (uint64_t)ii), ii, m);
        const float a = t[spp + j * m + ii], b = t[spp + j * m + k];
        t[spp + j * m + ii] = b;
        t[spp + j * m + k] = a;
      }
    }
  }
  return tb;
}

// The end of a work item: the pixel sums over the pixel's lanes, divided by
// the sample count (renderer.nim:159) and stored (renderer.nim:204-209: one
// pixel, or the step x step block of a progressive pass).
__device__ __forceinline__ void finish_item(KP p, const GroupPix& gp, F3 acc, int L) {
  if (L == 64) {  // one pixel per wave: DPP row scans + row broadcasts, total in lane 63
    acc = f3(wave_total(acc.x), wave_total(acc.y), wave_total(acc.z));
  } else {
    // the xor butterfly over the pixel's L lanes; inside a 16-lane row it is
    // DPP (quad_perm 1,0,3,2 / 2,3,0,1, row_ror:12 = lane i + 4, row_ror:8):
    // lane sub == 0 adds the butterfly's partners in its order, so its sum is
    // bit-identical (the other lanes' sums are not used)
    if (L >= 2) acc = f3(dpp_add<0xB1, 0xf>(acc.x), dpp_add<0xB1, 0xf>(acc.y), dpp_add<0xB1, 0xf>(acc.z));
    if (L >= 4) acc = f3(dpp_add<0x4E, 0xf>(acc.x), dpp_add<0x4E, 0xf>(acc.y), dpp_add<0x4E, 0xf>(acc.z));
    if (L >= 8) acc = f3(dpp_add<0x12C, 0xf>(acc.x), dpp_add<0x12C, 0xf>(acc.y), dpp_add<0x12C, 0xf>(acc.z));
    if (L >= 16) acc = f3(dpp_add<0x128, 0xf>(acc.x), dpp_add<0x128, 0xf>(acc.y), dpp_add<0x128, 0xf>(acc.z));
    for (int off = 16; off < L; off <<= 1) {
      acc.x += __shfl_xor(acc.x, off);
      acc.y += __shfl_xor(acc.y, off);
      acc.z += __shfl_xor(acc.z, off);
    }
  }
  if (gp.valid && gp.sub == 0) {
    if (p->aa_kind != 0) acc = f3(acc.x * p->inv_len, acc.y * p->inv_len, acc.z * p->inv_len);
    if (p->mode == 0 && p->step > 1) {
      // (every field re-read here: the progressive fill is rare, and operands
      // kept from the test above stayed live across the caller's item loop)
      p = params();
      const int xe = min(gp.x + p->step, p->width), ye = min(gp.y + p->step, p->height);
      for (int yy = gp.y; yy < ye; ++yy)
        for (int xx = gp.x; xx < xe; ++xx) {
          float* q = p->fb + ((size_t)yy * p->width + xx) * 3;
          q[0] = acc.x; q[1] = acc.y; q[2] = acc.z;
        }
    } else {
      float* q = p->fb + ((size_t)gp.out_row * p->width + gp.x) * 3;
      q[0] = acc.x; q[1] = acc.y; q[2] = acc.z;
    }
  }
}

// k_render_fast's item order: shard k hands out runs of RTMI_FAST_RUN
// consecutive pixel groups (k, k + shards, ... in runs), so a run of tiles —
// 32 pixels of a row for the 2 x 2 tiles of a 16-lane-per-pixel launch, i.e.
// three whole 128-B framebuffer lines — is written by waves of ONE XCD (the
// shard's blocks, blockIdx % shards), and a shard's waves share its pixels'
// object masks in their XCD's L2. Scheduling only (C2: 0.805 -> 0.794 ms,
// HBM 213 -> 87 MB per call).
#ifndef RTMI_FAST_RUN
#define RTMI_FAST_RUN 16
#endif
__device__ __forceinline__ int fast_item(int qj, int shards, int shard) {
  return (qj / RTMI_FAST_RUN * shards + shard) * RTMI_FAST_RUN + qj % RTMI_FAST_RUN;
}

template <bool COUNT, unsigned F>
// (the instrumented COUNT launch — bench.py's one traversal-counting call —
// carries more counters: 4 waves per SIMD keeps it spill-free too)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(COUNT ? 4u : waves_per_eu<F>()))) void
k_render_fast(const FastParams params_by_value) {
  (void)params_by_value;  // read through params() (kernarg segment)
  KP p = params();
  __shared__ float lds[4][kLdsSlots][64];            // 4 waves per 256-thread block
  extern __shared__ float sample_lds[];              // (multi-)jittered tables, sized by the host
  __shared__ unsigned long long lds_tot[4][kStatSlots];  // per-wave 64-bit Stats totals
  const int wib = (int)(threadIdx.x >> 6);
  LdsF* ls = (LdsF*)&lds[wib][0][__lane_id()];
  if (__lane_id() < (unsigned)kStatSlots) lds_tot[wib][__lane_id()] = 0ull;
  Stats32 ws;
#pragma unroll
  for (int k = 0; k < kStatSlots; ++k) ws.v[k] = 0u;

  // Work queue: the grid is exactly the resident waves (host: occupancy
  // query) and each wave pulls one work item at a time (coarser chunks left
  // an expensive tail in every launch). One head word saturates near 90
  // dequeues/us, so the heads are sharded 8 ways, one per blockIdx % 8 label
  // (blocks sharing an XCD; fewer shards when the grid has fewer than 8
  // blocks, so every shard has pullers), each on its own 128-B line; shard k
  // hands out items k, k+8, k+16, ... so every shard's work spans the whole
  // image. The next index is fetched one item ahead, hiding the atomic's
  // latency behind the samples. Item g is pixel group order[g] when the
  // host supplies an expensive-first order; a measuring launch records each
  // group's duration in cost[] (rtmi.cpp group_order).
  const int shard = (int)(blockIdx.x % (unsigned int)p->shards);
  unsigned int* head = p->queue + shard * kQueueStride;
  int qj = 0;
  if (__lane_id() == 0) qj = (int)atomicAdd(head, 1u);
  qj = __builtin_amdgcn_readfirstlane(qj);
  // reservations RTMI_QUEUE_AHEAD items ahead (lane 0 holds them): the
  // atomic's round trip overlaps that many items
  int qj_next = 0;
  if (__lane_id() == 0) qj_next = (int)atomicAdd(head, 1u);
#if RTMI_QUEUE_AHEAD >= 2
  int qj_next2 = 0;
  if (__lane_id() == 0) qj_next2 = (int)atomicAdd(head, 1u);
#endif
  int g = fast_item(qj, p->shards, shard);
  int nflush = 0;
  const int ngroups = list_items(p->list_n, p->ngroups, 1);
  while (g < ngroups) {
    p = params();
    const int L = p->lanes_per_px;
    const int iters = p->iters;
    const int gg = p->order ? cp(p->order)[g] : g;
    const unsigned t_item = (unsigned)__builtin_amdgcn_s_memtime();
    RT_STAMP(t_it0);
    const GroupPix gp = group_pixel(p, gg, lane_id_fresh());
    // multiJittered / correlatedMultiJittered (sampling.nim:39-113): the
    // wave builds each of its pixels' (m, m) tables in LDS — canonical
    // entries spread over the pixel's lanes, then the x shuffle with one
    // lane per column and the y shuffle with one lane per row (each lane
    // only touches its own column / row, so the sequential reference order
    // holds per lane; rt_sampling.h draw indices)
    LdsF* tb = sample_table<F>(p, gp, sample_lds, wib, L);
    Acc pacc;
    pacc.v = f3(0.0f, 0.0f, 0.0f);
    // the pixel's record, once per work item (a one-pixel wave: every
    // iteration shades the same pixel): list length + shadow skip bits. The
    // record speaks for every ray through the pixel's square grown by
    // rt_bins.h kPixelMargin, i.e. for sample offsets in [0, 1): the host
    // hands records (and pixel lists) only to samplers with that property
    // (rtmi.cpp sampler_in_pixel)
    unsigned pinfo = kPixCount;
    if ((F & F_MESH) && p->pix_info) {
      const unsigned long long vm = bal(gp.valid);
      if (vm != 0ull) {
        const int up = __builtin_amdgcn_readlane(gp.y * p->width + gp.x, (int)__builtin_ctzll(vm));
        pinfo = at(p->pix_info, up);
      }
    }
    // the per-sample loop; its LEAN instance is compiled without any mesh
    // search (below)
    auto sample_loop = [&](auto lean, int it_begin) {
      for (int it = it_begin; it < iters; ++it) {
        if (!decltype(lean)::value) p = params();
        const int s = it * L + gp.sub;  // this lane's sample index
        const bool sv = gp.valid & (s < p->spp);
        const F3 d = camera_dir<F>(p, gp, s < p->spp ? s : 0, tb);
        const F3 o = f3(p->cam[0], p->cam[1], p->cam[2]);
        ws.v[STAT_PRIMARY] += pc(bal(sv));
        RT_STAMP(t_s0);
        shade_path<COUNT, F, decltype(lean)::value>(p, o, d, sv, sv ? gp.y * p->width + gp.x : -1, pinfo, ls, pacc, ws);
#if RTMI_STAMPS == 1
        { RT_STAMP(t_s1); RT_ACC(7, t_s0, t_s1); }
#endif
      }
    };
    const int nlt = p->nlight;
    if ((F & F_MESH) && !(F & F_REFLECT) && (pinfo & kPixCount) == 0u && nlt <= 8 &&
        !((F & F_POINT) && p->has_point_light) &&
        ((pinfo >> 24) & ((1u << nlt) - 1u)) == (1u << nlt) - 1u) {
      // a lean pixel (no camera ray can hit the mesh, every light's shadow
      // rays skip it; no reflection): batches of samples per lane, then
      // the remaining iterations one at a time — both compiled without any
      // mesh search
      int it = 0;
#ifndef RTMI_NO_LEAN_BATCH
      for (; it + kLeanBatch <= iters; it += kLeanBatch) lean_batch<F>(p, gp, it, tb, pacc, ws);
#endif
      if (it < iters) sample_loop(Bool<true>{}, it);
    } else if constexpr (!(F & (F_MESH | F_REFLECT | F_POINT)) && (F & (F_SPHERE | F_BOX)) != 0) {
      // analytic scenes with distant lights (C2): object-binned batches —
      // kObjBatch samples per lane through the wave's pixels' object masks
      // and the shadow rays' light-grid cell masks, so each object visit's
      // scalar work (record load, dispatch, loop control) serves 64 x
      // kObjBatch rays; the remaining iterations one sample at a time
      unsigned long long cmask = p->nobj >= 64 ? ~0ull : ((1ull << p->nobj) - 1ull);
      if (p->obj_pix) {
        const int pix = gp.valid ? gp.y * p->width + gp.x : -1;
        if (L >= 8) {
          // <= 8 pixels per wave, pixel q's lanes from q L: every lane loads
          // its own pixel's mask (one vector load, one round trip for the
          // wave's pixels) and the pixels' first lanes are ORed — instead of
          // one scalar load per distinct pixel, each waited for in turn
          const unsigned long long mine = pix >= 0 ? p->obj_pix[pix] : 0ull;
          unsigned long long m = 0ull;
          for (int q = 0; q < 64; q += L)
            m |= ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)(mine >> 32), q) << 32) |
                 (unsigned)__builtin_amdgcn_readlane((int)(unsigned)mine, q);
          cmask = m;
        } else {
          unsigned long long todo = bal(pix >= 0), m = 0ull;
          for (int k = 0; k < 8 && todo != 0ull; ++k) {
            const int kp = __builtin_amdgcn_readlane(pix, (int)__builtin_ctzll(todo));
            todo &= ~bal(pix == kp);
            m |= cp(p->obj_pix)[kp];
          }
          cmask = todo == 0ull ? m : cmask;
        }
      }
      int it = 0;
      if (!(p->flags & RT_DEV_FLAG_NO_OBJ_BATCH))
        for (; it + kObjBatch <= iters; it += kObjBatch) lean_batch<F, kObjBatch, true>(p, gp, it, tb, pacc, ws, cmask);
      if (it < iters) sample_loop(Bool<false>{}, it);
    } else {
      sample_loop(Bool<false>{}, 0);
    }
    p = params();
    const int lane = lane_id_fresh();
    finish_item(p, gp, pacc.v, L);
    if (p->cost && lane == 0) p->cost[gg] = (unsigned)__builtin_amdgcn_s_memtime() - t_item;
#if RTMI_STAMPS == 1
    { RT_STAMP(t_it1); RT_ACC(8, t_it0, t_it1); }
#endif
    // 32-bit wave counters -> the wave's 64-bit LDS totals, every
    // p->stat_flush items (before any counter can wrap) and at the end
    if (++nflush >= p->stat_flush) {
      flush_stats(ws, lds_tot[wib], lane);
      nflush = 0;
    }
    qj = __builtin_amdgcn_readfirstlane(qj_next);
#if RTMI_QUEUE_AHEAD >= 2
    qj_next = qj_next2;
    if (lane == 0) qj_next2 = (int)atomicAdd(head, 1u);
#else
    if (lane == 0) qj_next = (int)atomicAdd(head, 1u);
#endif
    g = fast_item(qj, p->shards, shard);
  }
  p = params();
  const int lane = (int)__lane_id();
  flush_stats(ws, lds_tot[wib], lane);
  const int wave = (int)(blockIdx.x * (blockDim.x >> 6) + threadIdx.x / 64u);
  if (lane < kStatSlots) p->partials[(size_t)wave * kStatSlots + lane] = lds_tot[wib][lane];
}

// Reflection rays compacted per wave (renderer.nim:104-124; scenes with
// reflective materials). In k_render_fast a reflected ray is traced by the
// lane that shot its camera ray, one level per loop trip, so a level runs
// with only the wave's reflecting lanes live (spheres-reflection at 1080p:
// 20-40 % of a level-1 wave, fewer below). Here a camera iteration shades
// level 0 only; its reflected rays are appended (ballot + mbcnt ranks) to the
// wave's ray queue, which lives across work items, and whenever 64 rays are
// waiting they are shaded as one full pass — their own reflections appended
// again — so secondary levels, and the shadow rays they shoot, run with
// every lane live. The queue drains when the wave's work runs out.
//
// A queued ray's radiance belongs to a pixel the wave may have finished: it
// is added, as 32.32 fixed point, into the call's per-pixel secondary
// buffer (p->sec; integer sums are exact, so the frame does not depend on
// which rays shared a pass); k_sec_add adds it to the framebuffer after the
// kernel. A ray's level radiance is the same shade_level value as in
// k_render_fast; the pixel's sum is grouped differently (level 0 summed in
// float, the deeper levels in fixed point), so frames match k_render_fast's
// to float rounding and the Stats exactly.
//
// The queue is in global memory (L2-resident, kReflQueue x kReflFields
// floats per wave): in LDS its 4 KB per wave would cut the 8 resident waves
// per SIMD of the analytic reflective kernels to 5.
__device__ __forceinline__ long long sec_fix(float v) { return __float2ll_rn(v * 4294967296.0f); }
__device__ __forceinline__ long long wave_sum_i64(long long v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const unsigned lo = (unsigned)__shfl_xor((int)(unsigned)v, off);
    const unsigned hi = (unsigned)__shfl_xor((int)(unsigned)((unsigned long long)v >> 32), off);
    v += (long long)(((unsigned long long)hi << 32) | lo);
  }
  return v;
}
// A pass's radiance into p->sec: lanes sharing a destination pixel (high
// spp: a pass is mostly one or two pixels' rays) are summed in the wave
// first, one atomic per channel; scattered destinations add per lane.
__device__ __forceinline__ void sec_add(KP p, bool act, int dst, F3 v) {
  const long long c0 = sec_fix(v.x), c1 = sec_fix(v.y), c2 = sec_fix(v.z);
  const bool any = act && (c0 | c1 | c2) != 0;
  unsigned long long pend = bal(any);
  const int lane = lane_id_fresh();
  long long* sec = p->sec - p->sec_base * 3;
  for (int k = 0; k < 4 && pend != 0ull; ++k) {
    const int lead = (int)__builtin_ctzll(pend);
    const int d0 = __builtin_amdgcn_readlane(dst, lead);
    const bool mine = any && dst == d0;
    const unsigned long long mm = bal(mine);
    if (pc(mm) < 4u) break;  // scattered: per lane below
    pend &= ~mm;
    const long long s0 = wave_sum_i64(mine ? c0 : 0), s1 = wave_sum_i64(mine ? c1 : 0),
                    s2 = wave_sum_i64(mine ? c2 : 0);
    if (lane == lead) {
      long long* q = sec + (size_t)d0 * 3;
      atomicAdd((unsigned long long*)q + 0, (unsigned long long)s0);
      atomicAdd((unsigned long long*)q + 1, (unsigned long long)s1);
      atomicAdd((unsigned long long*)q + 2, (unsigned long long)s2);
    }
  }
  if ((pend >> lane) & 1ull) {
    long long* q = sec + (size_t)dst * 3;
    atomicAdd((unsigned long long*)q + 0, (unsigned long long)c0);
    atomicAdd((unsigned long long*)q + 1, (unsigned long long)c1);
    atomicAdd((unsigned long long*)q + 2, (unsigned long long)c2);
  }
}
// queue entries: read back with device-scope loads (they bypass the CU's
// L1, which may hold an older copy of the slot), after the wave's stores
// have completed (the release fence)
__device__ __forceinline__ float rq_load(const float* q) {
  return __uint_as_float(__hip_atomic_load((const unsigned*)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

template <unsigned F>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(wave_waves<F>()))) void k_render_wave(
    const FastParams params_by_value) {
  static_assert(F & F_REFLECT, "the compacting kernel serves reflective scenes");
  (void)params_by_value;
  KP p = params();
  __shared__ float lds[4][kLdsSlots][64];
  extern __shared__ float sample_lds[];
  __shared__ unsigned long long lds_tot[4][kStatSlots];
  const int wib = (int)(threadIdx.x >> 6);
  LdsF* ls = (LdsF*)&lds[wib][0][__lane_id()];
  if (__lane_id() < (unsigned)kStatSlots) lds_tot[wib][__lane_id()] = 0ull;
  Stats32 ws;
#pragma unroll
  for (int k = 0; k < kStatSlots; ++k) ws.v[k] = 0u;
  const int wave = (int)(blockIdx.x * (blockDim.x >> 6) + threadIdx.x / 64u);
  float* const rq = p->rq + (size_t)wave * (kReflQueue * kReflFields);
  // work queue as in k_render_fast (sharded heads, one item ahead)
  const int shard = (int)(blockIdx.x % (unsigned int)p->shards);
  unsigned int* head = p->queue + shard * kQueueStride;
  int qj = 0;
  if (__lane_id() == 0) qj = (int)atomicAdd(head, 1u);
  qj = __builtin_amdgcn_readfirstlane(qj);
  int qj_next = 0;
  if (__lane_id() == 0) qj_next = (int)atomicAdd(head, 1u);
  int g = qj * p->shards + shard;
  const int ngroups = list_items(p->list_n, p->ngroups, 1);
  int nflush = 0, qn = 0, it = 0, gg = 0;
  bool have = false;
  unsigned t_item = 0u, pinfo = kPixCount;
  GroupPix gp{};
  LdsF* tb = nullptr;
  Acc pacc;
  pacc.v = f3(0.0f, 0.0f, 0.0f);
  auto next_item = [&]() {
    have = g < ngroups;
    if (!have) return;
    p = params();
    gg = p->order ? cp(p->order)[g] : g;
    t_item = (unsigned)__builtin_amdgcn_s_memtime();
    gp = group_pixel(p, gg, lane_id_fresh());
    tb = sample_table<F>(p, gp, sample_lds, wib, p->lanes_per_px);
    pacc.v = f3(0.0f, 0.0f, 0.0f);
    it = 0;
    pinfo = kPixCount;
    if ((F & F_MESH) && p->pix_info) {
      const unsigned long long vm = bal(gp.valid);
      if (vm != 0ull) pinfo = at(p->pix_info, __builtin_amdgcn_readlane(gp.y * p->width + gp.x, (int)__builtin_ctzll(vm)));
    }
    qj = __builtin_amdgcn_readfirstlane(qj_next);
    if (__lane_id() == 0) qj_next = (int)atomicAdd(head, 1u);
    g = qj * p->shards + shard;
  };
  next_item();
  for (;;) {
    p = params();
    if (have && it >= p->iters) {  // the item's camera samples are all shaded
      finish_item(p, gp, pacc.v, p->lanes_per_px);
      if (p->cost && lane_id_fresh() == 0) p->cost[gg] = (unsigned)__builtin_amdgcn_s_memtime() - t_item;
      if (++nflush >= p->stat_flush) {
        flush_stats(ws, lds_tot[wib], lane_id_fresh());
        nflush = 0;
      }
      next_item();
      continue;
    }
    const bool from_q = qn >= 64 || (!have && qn > 0);
    if (!from_q && !have) break;
    const int lane = lane_id_fresh();
    F3 o, d;
    bool act;
    float w;
    int depth, dst, lev;
    if (from_q) {  // a pass over the newest min(qn, 64) queued rays
      const int n = min(qn, 64);
      qn -= n;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      act = lane < n;
      const float* e = rq + qn + (act ? lane : 0);
      o = f3(rq_load(e + 0 * kReflQueue), rq_load(e + 1 * kReflQueue), rq_load(e + 2 * kReflQueue));
      d = f3(rq_load(e + 3 * kReflQueue), rq_load(e + 4 * kReflQueue), rq_load(e + 5 * kReflQueue));
      w = rq_load(e + 6 * kReflQueue);
      const int meta = __float_as_int(rq_load(e + 7 * kReflQueue));
      dst = meta >> 4;
      depth = meta & 15;
      lev = 1;
    } else {  // the item's next camera iteration: level 0 of its samples
      const int s = it * p->lanes_per_px + gp.sub;
      act = gp.valid & (s < p->spp);
      d = camera_dir<F>(p, gp, s < p->spp ? s : 0, tb);
      o = f3(p->cam[0], p->cam[1], p->cam[2]);
      ws.v[STAT_PRIMARY] += pc(bal(act));
      w = 1.0f;
      depth = 1;
      dst = gp.out_row * p->width + gp.x;
      lev = 0;
      ++it;
    }
    F3 v;
    bool reflect;
    float refl;
    shade_level<false, F, false>(p, o, d, act, lev, depth, w, lev == 0 && act ? gp.y * p->width + gp.x : -1, pinfo,
                                 ls, v, reflect, refl, ws);
    p = params();
    if (lev == 0) {
      if (act) acc_add3(pacc, v.x, v.y, v.z);
    } else {
      sec_add(p, act, dst, v);
    }
    const unsigned long long rm = bal(reflect);
    if (rm != 0ull) {  // append the reflected rays (parked in LDS by shade_level)
      if (reflect) {
        const int slot = qn + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(rm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)rm, 0u));
        const F3 ro = lds_get3(ls, LDS_RO), rd = lds_get3(ls, LDS_RD);
        float* e = rq + slot;
        e[0 * kReflQueue] = ro.x;
        e[1 * kReflQueue] = ro.y;
        e[2 * kReflQueue] = ro.z;
        e[3 * kReflQueue] = rd.x;
        e[4 * kReflQueue] = rd.y;
        e[5 * kReflQueue] = rd.z;
        e[6 * kReflQueue] = w * refl;
        e[7 * kReflQueue] = __int_as_float(dst * 16 + depth + 1);
      }
      qn += (int)pc(rm);
    }
  }
  p = params();
  const int lane = (int)__lane_id();
  flush_stats(ws, lds_tot[wib], lane);
  if (lane < kStatSlots) p->partials[(size_t)wave * kStatSlots + lane] = lds_tot[wib][lane];
}

// The lean-pixel kernel (two-class launches, rtmi.cpp split_lists): the
// work items are the launch's lean pixel groups (p->order lists them,
// p->ngroups counts them), every one rendered by lean_batch. The kernel
// holds nothing but that path, so unlike k_render_fast (whose register
// allocation is set by the mesh searches: kernel arguments re-read per use,
// spilled SGPRs) its item loop keeps the arguments in SGPRs; per work item
// it costs a dequeue, a list read and the pixel sum. Frames are
// bit-identical to k_render_fast's lean path (same lean_batch, same sums).
#ifndef RTMI_LEAN_WAVES
#define RTMI_LEAN_WAVES 8
#endif
template <unsigned F>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(occ_table<F>(kOcc_lean, RTMI_LEAN_WAVES)))) void
k_render_lean(
    const FastParams params_by_value) {
  (void)params_by_value;
  const KP p = params();
  extern __shared__ float sample_lds[];
  __shared__ unsigned long long lds_tot[4][kStatSlots];
  const int wib = (int)(threadIdx.x >> 6);
  const int lane = (int)__lane_id();
  if (lane < kStatSlots) lds_tot[wib][lane] = 0ull;
  Stats32 ws;
#pragma unroll
  for (int k = 0; k < kStatSlots; ++k) ws.v[k] = 0u;
  const int shard = (int)(blockIdx.x % (unsigned int)p->shards);
  unsigned int* head = p->queue + shard * kQueueStride;
  int qj = 0;
  if (lane == 0) qj = (int)atomicAdd(head, 1u);
  qj = __builtin_amdgcn_readfirstlane(qj);
  int qj_next = 0;
  if (lane == 0) qj_next = (int)atomicAdd(head, 1u);
  int g = qj * p->shards + shard;
  int nflush = 0;
  const int iters = p->iters;
  // a work item is a run of kLeanRun list entries (p->ngroups counts runs;
  // the host pads the list with -1): one dequeue and one scalar load per
  // run, and the next run's entries are loaded while this run renders (the
  // per-item dequeue + dependent list read measured ~40 % of an all-lean
  // frame with one pixel per item)
  static_assert(kLeanRun == 4, "a run is one s_load_dwordx4");
  using Run = int32_t __attribute__((ext_vector_type(4)));
  const RT_CONST Run* runs = (const RT_CONST Run*)cp(p->order);
  const int nruns = list_items(p->list_n, p->ngroups, kLeanRun);
  Run ent = g < nruns ? runs[g] : Run{-1, -1, -1, -1};
  while (g < nruns) {
    qj = __builtin_amdgcn_readfirstlane(qj_next);
    if (lane == 0) qj_next = (int)atomicAdd(head, 1u);
    const int gn = qj * p->shards + shard;
    const Run ent_next = gn < nruns ? runs[gn] : Run{-1, -1, -1, -1};
#pragma unroll 1
    for (int r = 0; r < kLeanRun; ++r) {
      const int gg = ent.x;  // the entries shift down (static swizzles, no indexed SGPR access)
      ent = Run{ent.y, ent.z, ent.w, -1};
      if (gg < 0) break;  // padding: the list's last run
      GroupPix gp = group_pixel(p, gg, lane);
      gp.valid = true;  // the lists hold only pixels of the launch (rtmi.cpp split_lists)
      const LdsF* tb = sample_table<F>(p, gp, sample_lds, wib, 64);
      Acc acc;
      acc.v = f3(0.0f, 0.0f, 0.0f);
      int it = 0;
      for (; it + kLeanBatch <= iters; it += kLeanBatch) lean_batch<F, kLeanBatch>(p, gp, it, tb, acc, ws);
      for (; it < iters; ++it) lean_batch<F, 1>(p, gp, it, tb, acc, ws);
      finish_item(p, gp, acc.v, 64);
    }
    if (++nflush >= p->stat_flush) {
      flush_stats(ws, lds_tot[wib], lane);
      nflush = 0;
    }
    ent = ent_next;
    g = gn;
  }
  flush_stats(ws, lds_tot[wib], lane);
  const int wave = (int)(blockIdx.x * (blockDim.x >> 6) + threadIdx.x / 64u);
  if (lane < kStatSlots) p->partials[(size_t)wave * kStatSlots + lane] = lds_tot[wib][lane];
}

// Lean pixels of a scene whose only analytic object is one plane (C3-C5: the
// mesh on a ground plane), every transform a translation, NL distant lights
// (1 or 2), akGrid with m | 64 and spp a multiple of 64 (every sample valid,
// a lane's samples share one column) — rtmi.cpp lean1_ok decides. The same
// per-sample arithmetic as lean_batch's uniform single-plane case, with what
// that case leaves wave-uniform or per lane formed once:
//  * the camera ray needs only its y direction (the plane test, the hit
//    point's height); the cx terms of camera_ray_dir are per lane and pixel;
//  * a plane's normal is (0, 1, 0), so every lit sample of the pixel has the
//    same N, N.L per light and albedo: shadeDiffuse's term per light is one
//    select of a uniform value, the colour lit ? albedo x E : background;
//  * "t >= 0 and below the running limit" is, against a first (and only)
//    object, one class test of t (finite, >= 0 incl. -0);
//  * sample validity, object dispatch, the mesh skip and the per-object
//    loops are gone (one plane, all samples valid).
// Frames and Stats bit-identical to k_render_lean / k_render_fast
// (tests/test_gpu_split.py, RT_FLAG_NO_LEAN1).
// "t >= 0 and below the running limit" against a first object (limit
// +inf): t in [-0, +inf), NaN excluded.
// One v_cmp_class straight into a lane mask: classes -0, +0, +denormal,
// +normal (the kernels run with fp32 denormals preserved,
// .amdhsa_float_denorm_mode_32 3, so compares see denormals as such). The
// builtin's bool went through a VGPR and back (v_cndmask + v_cmp).
__device__ __forceinline__ unsigned long long m_hit0(float t) {
  unsigned long long m;
  asm("v_cmp_class_f32_e64 %0, %1, %2" : "=s"(m) : "v"(t), "v"(0x1E0));
  return m;
}
template <int NL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_render_lean1(
    const FastParams params_by_value) {
  (void)params_by_value;
  constexpr int S = 4;  // samples per lane per batch: the host requires iters % 4 == 0
  const KP p = params();
  __shared__ unsigned long long lds_tot[4][kStatSlots];
  const int wib = (int)(threadIdx.x >> 6);
  const int lane = (int)__lane_id();
  if (lane < kStatSlots) lds_tot[wib][lane] = 0ull;
  Stats32 ws;
#pragma unroll
  for (int k = 0; k < kStatSlots; ++k) ws.v[k] = 0u;
  const int shard = (int)(blockIdx.x % (unsigned int)p->shards);
  unsigned int* head = p->queue + shard * kQueueStride;
  int qj = 0;
  if (lane == 0) qj = (int)atomicAdd(head, 1u);
  qj = __builtin_amdgcn_readfirstlane(qj);
  int qj_next = 0;
  if (lane == 0) qj_next = (int)atomicAdd(head, 1u);
  int g = qj * p->shards + shard;
  int nflush = 0;
  const int iters = p->iters;
  // the scene's one analytic object (the other is the mesh): a plane whose
  // world -> object transform is a translation
  const int po = p->shadow_mesh == 0 ? 1 : 0;
  const FObj pl = at(p->objs, po);
  const RT_CONST FObjX& plx = at(p->objx, po);
  const float nroy = -(p->cam[1] + pl.t[1]);  // -(camera origin in plane space).y: Plane.intersect's -o.y
  const float ty = pl.t[1], oy = p->cam[1], bias = p->bias;
  // per light: the parallel shadow rays' plane reciprocal (a NaN multiplier
  // when parallel: no t >= 0), N.L with N = (0, 1, 0) (dot3's roundings), ci
  float mulp[NL], ndl[NL], ci[NL][3];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    const FLight L = at(p->lights, l);
    const F3 sd = f3(-L.v[0], -L.v[1], -L.v[2]);
    mulp[l] = fabsf(sd.y) > 1e-6f ? rcp(sd.y) : __builtin_nanf("");
    ndl[l] = fmaxf(dot3(f3(0.0f, 1.0f, 0.0f), sd), 0.0f);
    ci[l][0] = L.ci[0];
    ci[l][1] = L.ci[1];
    ci[l][2] = L.ci[2];
  }
  const F3 alb = f3(plx.albedo_pi[0], plx.albedo_pi[1], plx.albedo_pi[2]);
  const F3 bg = f3(p->bg[0], p->bg[1], p->bg[2]);
  const int mm = p->grid_m - 1, lg = p->log2_grid_m;
  const float st = p->sample_step, of = p->sample_off;
  static_assert(kLeanRun == 4, "a run is one s_load_dwordx4");
  using Run = int32_t __attribute__((ext_vector_type(4)));
  const RT_CONST Run* runs = (const RT_CONST Run*)cp(p->order);
  const int nruns = list_items(p->list_n, p->ngroups, kLeanRun);
  Run ent = g < nruns ? runs[g] : Run{-1, -1, -1, -1};
  while (g < nruns) {
    qj = __builtin_amdgcn_readfirstlane(qj_next);
    if (lane == 0) qj_next = (int)atomicAdd(head, 1u);
    const int gn = qj * p->shards + shard;
    const Run ent_next = gn < nruns ? runs[gn] : Run{-1, -1, -1, -1};
#pragma unroll 1
    for (int r = 0; r < kLeanRun; ++r) {
      const int gg = ent.x;
      ent = Run{ent.y, ent.z, ent.w, -1};
      if (gg < 0) break;
      GroupPix gp = group_pixel(p, gg, lane);
      gp.valid = true;
      // the lane's column: camera_ray_dir's cx terms, once per pixel
      const float px = (float)gp.x + __builtin_fmaf((float)(gp.sub & mm), st, of);
      const float cx = (px - p->cam_b) * p->cam_a;
      const float q0 = __builtin_fmaf(cx, cx, 1.0f);
      const float ay = __builtin_fmaf(cx, p->cam[4], -p->cam[10]);
      const float pyb = (float)gp.y;
      Acc acc;
      acc.v = f3(0.0f, 0.0f, 0.0f);
      unsigned nlit = 0u, nocc = 0u;
#pragma unroll 1
      for (int it0 = 0; it0 < iters; it0 += S) {
        float soy[S];
        unsigned long long litm[S];
#pragma unroll
        for (int k = 0; k < S; ++k) {
          // castPrimaryRay's direction, y only; Plane.intersect; trace's rule
          const int s = (it0 + k) * 64 + gp.sub;
          const float py = pyb + __builtin_fmaf((float)(s >> lg), st, of);
          const float cy = (p->cam_d - py) * p->cam_c;
          const float rl = rsq(__builtin_fmaf(cy, cy, q0));
          const float dy = __builtin_fmaf(cy, p->cam[7], ay) * rl;
          const float t = fabsf(dy) > 1e-6f ? nroy * rcp(dy) : -finf();
          litm[k] = m_hit0(t);  // the camera ray hits the plane: a hit, and a lit sample
          nlit += pc(litm[k]);
          // the shadow origin's height: hitW.y + N.y * bias (N.y = 1)
          soy[k] = __builtin_fmaf(1.0f, bias, __builtin_fmaf(dy, t, oy));
        }
#pragma unroll
        for (int k = 0; k < S; ++k) {
          const bool lit = lane_in(litm[k]);
          F3 E = f3(0.0f, 0.0f, 0.0f);
#pragma unroll
          for (int l = 0; l < NL; ++l) {
            const float ts = -(soy[k] + ty) * mulp[l];
            const unsigned long long occ = m_hit0(ts) & litm[k];  // the shadow ray hits the plane
            nocc += pc(occ);
            const float x = lane_in(litm[k] & ~occ) ? ndl[l] : 0.0f;
            E = f3(__builtin_fmaf(ci[l][0], x, E.x), __builtin_fmaf(ci[l][1], x, E.y),
                   __builtin_fmaf(ci[l][2], x, E.z));
          }
          const F3 a = mul3(alb, E);
          acc_add3(acc, lit ? a.x : bg.x, lit ? a.y : bg.y, lit ? a.z : bg.z);
        }
      }
      ws.v[STAT_PRIMARY] += (unsigned)(64 * iters);
      ws.v[STAT_SHADOW] += (unsigned)NL * nlit;
      ws.v[STAT_HITS] += nlit + nocc;  // camera hits (= lit samples) + shadow hits
      finish_item(p, gp, acc.v, 64);
    }
    if (++nflush >= p->stat_flush) {
      flush_stats(ws, lds_tot[wib], lane);
      nflush = 0;
    }
    ent = ent_next;
    g = gn;
  }
  flush_stats(ws, lds_tot[wib], lane);
  const int wave = (int)(blockIdx.x * (blockDim.x >> 6) + threadIdx.x / 64u);
  if (lane < kStatSlots) p->partials[(size_t)wave * kStatSlots + lane] = lds_tot[wib][lane];
}

// Work queue of one list of n items over `shards` heads at `queue`; the
// blocks b with b % shards == s pull from head s, so shard s runs on XCD
// s % 8 (workgroups are dealt out to the 8 XCDs round robin).
// Default: shard s hands out runs of R consecutive items, s R .. s R + R - 1,
// then (s + S) R .., ... (every shard's items span the image; R = RUN: a run
// of neighbouring pixels is written by one XCD, so fewer framebuffer lines
// are written back partially by two XCDs' L2s). RTMI_XCD_CHUNK=1 (A/B only, measured slower: C3
// 0.93 -> 1.10 ms, rank 0 of 8 0.165 -> 0.396 ms — the bunny's expensive
// items fall into few chunks and the other XCDs end up stealing from one
// head): the list is cut into S contiguous chunks,
// chunk c = [c n / S, (c + 1) n / S), and the S / 8 shards of an XCD own
// consecutive chunks (shard s: chunk (s % 8) S / 8 + s / 8; S a multiple of
// 8, else chunk s) — the lists are in image tile order, so an XCD's waves
// work on one horizontal slab of the image and its L2 holds that slab's faces
// and cell lists. A wave whose chunk is exhausted moves on to the next chunk
// (the next shard of its XCD, at the slab's end the next XCD's first) and
// takes that chunk's next items, so no XCD idles while items remain; each
// wave visits every chunk at most once (the loop ends). The next
// reservation is fetched one item ahead (its atomic's latency hides behind
// the item).
#ifndef RTMI_XCD_CHUNK
#define RTMI_XCD_CHUNK 0
#endif
#ifndef RTMI_GEN_RUN
#define RTMI_GEN_RUN 8   // general items (one pixel each): 8 pixels = 96 B of framebuffer per run
#endif
#ifndef RTMI_LEAN_RUN
#define RTMI_LEAN_RUN 2  // one-plane lean items (4 or 16 pixels each)
#endif
template <int RUN = 1>
struct WorkQ {
  unsigned int* queue;
  int shards, n, cur, left, lo, len, qj_next, head;

  __device__ __forceinline__ void bounds() {
#if RTMI_XCD_CHUNK
    lo = (int)(((long long)cur * n) / shards);
    len = (int)(((long long)(cur + 1) * n) / shards) - lo;
    const int per = shards >> 3;  // chunks per XCD
    head = (shards & 7) == 0 ? (cur % per) * 8 + cur / per : cur;
#else
    head = cur;
    lo = cur;
    len = n;
#endif
  }
  // (scalar at once: the compiler's atomic optimizer already waits for the
  // atomic and reads its result with readfirstlane where it is issued, so a
  // per-lane copy bought no latency hiding — it only held a VGPR across the
  // item, which k_render_mix1 spilled)
  // RTMI_QSCALAR=0 (A/B): the per-lane copy again (with the atomic
  // optimiser off — Makefile F32_FLAGS — a true prefetch): C3 equal, one
  // spilled VGPR in k_render_mix1 (profiles/r5/ab/r5af_*)
#ifndef RTMI_QSCALAR
#define RTMI_QSCALAR 1
#endif
  __device__ __forceinline__ int reserve() {
    int q = 0;
    if (__lane_id() == 0) q = (int)atomicAdd(queue + head * kQueueStride, 1u);
    return RTMI_QSCALAR ? __builtin_amdgcn_readfirstlane(q) : q;
  }
  __device__ __forceinline__ int item(int qj) const {
#if RTMI_XCD_CHUNK
    return lo + qj;
#else
    return (qj / RUN * shards + lo) * RUN + qj % RUN;
#endif
  }
  __device__ __forceinline__ bool in(int qj) const {
#if RTMI_XCD_CHUNK
    return qj < len;
#else
    return item(qj) < n;
#endif
  }
  // the first item (-1: none)
  __device__ __forceinline__ int start(unsigned int* q, int s, int items) {
    queue = q;
    shards = s;
    n = items;
    const int shard = (int)(blockIdx.x % (unsigned int)s);
#if RTMI_XCD_CHUNK
    cur = (s & 7) == 0 ? (shard & 7) * (s >> 3) + (shard >> 3) : shard;
#else
    cur = shard;
#endif
    left = s;
    bounds();
    qj_next = reserve();
    return next();
  }
  // the next item (-1: every shard is exhausted)
  __device__ __forceinline__ int next() {
    for (;;) {
      const int qj = __builtin_amdgcn_readfirstlane(qj_next);
      if (in(qj)) {
        qj_next = reserve();
        return item(qj);
      }
#if RTMI_XCD_CHUNK
      if (--left <= 0) return -1;
      cur = cur + 1 == shards ? 0 : cur + 1;
      bounds();
      qj_next = reserve();
#else
      return -1;
#endif
    }
  }
};

// A one-pixel group's placement computed per lane (g differs per lane):
// group_pixel for tile 1 x 1 (lanes_per_px = 64), without the validity test
// (list entries are pixels of the launch).
__device__ __forceinline__ GroupPix lane_pixel(KP p, int g) {
  GroupPix r;
  r.sub = 0;
  r.valid = true;
  const int k = (int)(((unsigned long long)(unsigned)g * p->tx_magic) >> p->tx_shift);  // g / tiles_x
  const int j = g - k * p->tiles_x;
  r.x = j * p->step;
  if (p->mode == 0) {
    r.y = p->y0 + k * p->step;
    r.out_row = r.y;
  } else {
    int rr;
    const int lb = div_small(k, p->band_h, p->inv_band_h, rr);
    r.y = (lb * p->world + p->rank) * p->band_h + rr;
    r.out_row = k;
  }
  return r;
}

// The one-plane lean pixels with LP lanes per pixel (k_render_lean1's
// arithmetic per sample, a different assignment of samples to lanes): lane
// LP i + q of a wave renders "virtual lanes" V q .. V q + V - 1 (V = 64 / LP)
// of pixel i of a (64 / LP)-pixel work item — the samples k_render_lean1's
// lanes V q .. carry — each virtual lane's samples added in sample order as
// there, a lane's V virtual lanes in the balanced pairwise order of
// wave_total's DPP row scan (a binary-counter stack), then the lanes of the
// pixel pairwise by xor shuffles (1, 2, 4, 8, ...): wave_total is that
// balanced tree over the 64 lanes (row scans, then rows as ((R0 + R1) +
// (R2 + R3))). So every pixel is the same float sum as in k_render_lean1,
// bit for bit, with no per-pixel wave reduction and the per-pixel set-up
// spread over 64 / LP pixels at once. LP = 4 (16 pixels per item) for whole
// frames, 16 (4 per item) for short launches (rtmi.cpp).
// k_render_lean1q's work loop over one list (order: 64 / LP entries per
// item, ngroups items, dequeued from the shard heads at `queue`); also the
// second phase of k_render_mix1.
#ifndef RTMI_LEAN1Q_H
#define RTMI_LEAN1Q_H 1
#endif
template <int NL, int LP>
__device__ __forceinline__ void lean1q_loop(KP p, const int32_t* order, int ngroups, unsigned int* queue, int shards,
                                            Stats32& ws, unsigned long long* tot, int& nflush) {
  const int lane = (int)__lane_id();
  WorkQ<RTMI_LEAN_RUN> wq;
  int g = wq.start(queue, shards, ngroups);
  if (g < 0) return;
  const int iters = p->iters;
  const int po = p->shadow_mesh == 0 ? 1 : 0;
  const FObj pl = at(p->objs, po);
  const RT_CONST FObjX& plx = at(p->objx, po);
  const float nroy = -(p->cam[1] + pl.t[1]);
  const float ty = pl.t[1], oy = p->cam[1], bias = p->bias;
  float mulp[NL], ndl[NL], ci[NL][3];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    const FLight L = at(p->lights, l);
    const F3 sd = f3(-L.v[0], -L.v[1], -L.v[2]);
    mulp[l] = fabsf(sd.y) > 1e-6f ? rcp(sd.y) : __builtin_nanf("");
    ndl[l] = fmaxf(dot3(f3(0.0f, 1.0f, 0.0f), sd), 0.0f);
    ci[l][0] = L.ci[0];
    ci[l][1] = L.ci[1];
    ci[l][2] = L.ci[2];
  }
  const F3 alb = f3(plx.albedo_pi[0], plx.albedo_pi[1], plx.albedo_pi[2]);
  F3 bg = f3(p->bg[0], p->bg[1], p->bg[2]);
  // the background in VGPRs for the whole loop: a select against an SGPR
  // operand with the mask in VCC needs a v_mov per use (constant bus)
  asm volatile("" : "+v"(bg.x), "+v"(bg.y), "+v"(bg.z));
  const int mm = p->grid_m - 1, lg = p->log2_grid_m;
  const float st = p->sample_step, of = p->sample_off;
  static_assert(LP == 4 || LP == 8 || LP == 16, "lanes per pixel");
  constexpr int V = 64 / LP;   // virtual lanes per lane
  constexpr int H = RTMI_LEAN1Q_H;  // virtual lanes per step (independent sample chains)
  static_assert(H == 1 || H == 2, "one or two virtual lanes per step");
  constexpr int PPI = 64 / LP; // pixels per work item
  const int q = lane & (LP - 1);  // this lane's share of its pixel's virtual lanes
  // Every lit sample traces each light's shadow ray: against the plane here
  // (ts = -(soy + ty) m_l, a hit at ts in [0, +inf) occludes it), against the
  // mesh by the pixel's record — a lean pixel's skip bits, built this call
  // (rt_frame.hip k_frame_records), say that no shadow ray leaving a camera
  // hit of the pixel can meet a face of the mesh. When no lane's shadow ray
  // hits the plane for a sample (the usual case: lights above the plane), a
  // lit sample's colour is av = albedo x E over all lights — formed once here
  // in the per-light chain's order, so it is the value that chain gives.
  F3 av;
  {
    F3 E = f3(0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int l = 0; l < NL; ++l)
      E = f3(__builtin_fmaf(ci[l][0], ndl[l], E.x), __builtin_fmaf(ci[l][1], ndl[l], E.y),
             __builtin_fmaf(ci[l][2], ndl[l], E.z));
    av = mul3(alb, E);
  }
  asm volatile("" : "+v"(av.x), "+v"(av.y), "+v"(av.z));
  while (g >= 0) {
    const int gg = order[g * PPI + lane / LP];  // this lane's pixel (list entry; -1: padding)
    const unsigned long long vmask = bal(gg >= 0);
    const GroupPix gp = lane_pixel(p, gg >= 0 ? gg : 0);
    const float pxb = (float)gp.x, pyb = (float)gp.y;
    unsigned nlit = 0u, nocc = 0u;
    // the binary-counter stack of the V virtual lanes' partial sums, two
    // virtual lanes at a time (two independent sample chains per step; their
    // sum is the tree's first level)
    F3 s1 = f3(0.0f, 0.0f, 0.0f), s2 = s1, s3 = s1, sum = s1, s0 = s1;
    static_assert(V % 2 == 0, "virtual lanes in pairs");
    // the sample row of virtual lane jv in iteration it: (it * 64 + jv) >> lg
    // == it * (64 >> lg) + (jv >> lg) (m | 64), and jv >> lg == (q V) >> lg
    // for all of this lane's virtual lanes (m >= 16, rtmi.cpp lean1_ok, so V
    // divides 2^lg): one camera y per iteration for the whole lane, formed
    // from exact small-integer floats as k_render_lean1 steps them
    float rows = (float)(64 >> lg), sj0 = (float)((q * V) >> lg);
    // formed per item (opaque): hoisted out of the item loop, the four
    // per-lane row offsets below lived across every item and spilled
    asm volatile("" : "+v"(sj0));
    float cyc[4];  // the camera y of four consecutive iterations from it0
    auto cy_rows = [&](int it0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float py = pyb + __builtin_fmaf(__builtin_fmaf((float)(it0 + k), rows, sj0), st, of);
        cyc[k] = (p->cam_d - py) * p->cam_c;
      }
    };
    if (iters == 4) cy_rows(0);  // one chunk (m = 16): once per item
#pragma unroll 1
    for (int j = 0; j < V; j += H) {
      float q0[H], ay[H];
      F3 acc[H];
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const int jv = q * V + j + h;  // the virtual lane (k_render_lean1's lane)
        const float px = pxb + __builtin_fmaf((float)(jv & mm), st, of);
        const float cx = (px - p->cam_b) * p->cam_a;
        q0[h] = __builtin_fmaf(cx, cx, 1.0f);
        ay[h] = __builtin_fmaf(cx, p->cam[4], -p->cam[10]);
        acc[h] = f3(0.0f, 0.0f, 0.0f);
      }
      // iters is a multiple of 4 (rtmi.cpp lean1_ok): four samples per step
#pragma unroll 1
      for (int it0 = 0; it0 < iters; it0 += 4) {
      if (iters != 4) cy_rows(it0);
#pragma unroll
      for (int it = 0; it < 4; ++it)
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const float cy = cyc[it];
        const float rl = rsq(__builtin_fmaf(cy, cy, q0[h]));
        const float dy = __builtin_fmaf(cy, p->cam[7], ay[h]) * rl;
        // (|dy| <= 1e-6: no hit; t is only read on lit lanes)
        const float t = nroy * rcp(dy);
        const unsigned long long litm = m_hit0(t) & bal(fabsf(dy) > 1e-6f) & vmask;
        nlit += pc(litm);
        const bool lit = lane_in(litm);
        const float soy = __builtin_fmaf(1.0f, bias, __builtin_fmaf(dy, t, oy));
        unsigned long long occ[NL], any = 0ull;
#pragma unroll
        for (int l = 0; l < NL; ++l) {
          const float ts = -(soy + ty) * mulp[l];
          occ[l] = m_hit0(ts) & litm;
          nocc += pc(occ[l]);
          any |= occ[l];
        }
        F3 a = av;
        if (any != 0ull) {  // some shadow ray hit the plane: the per-light chain
          F3 E = f3(0.0f, 0.0f, 0.0f);
#pragma unroll
          for (int l = 0; l < NL; ++l) {
            const float x = lane_in(litm & ~occ[l]) ? ndl[l] : 0.0f;
            E = f3(__builtin_fmaf(ci[l][0], x, E.x), __builtin_fmaf(ci[l][1], x, E.y), __builtin_fmaf(ci[l][2], x, E.z));
          }
          a = mul3(alb, E);
        }
        acc[h] = f3(acc[h].x + (lit ? a.x : bg.x), acc[h].y + (lit ? a.y : bg.y), acc[h].z + (lit ? a.z : bg.z));
      }
      }
      // push the pair's sum: pair index P = j / 2 pairs with the stack while
      // it has trailing ones (uniform branches); one virtual lane per step
      // (H = 1): the even one waits in s0 for its odd partner (the same sum)
      F3 lo = acc[0], hi = acc[H - 1];
      if constexpr (H == 1) {
        if ((j & 1) == 0) {
          s0 = acc[0];
          continue;
        }
        lo = s0;
      }
      const int P = j >> 1;
      F3 t = f3(lo.x + hi.x, lo.y + hi.y, lo.z + hi.z);
      if (P & 1) {
        t = f3(s1.x + t.x, s1.y + t.y, s1.z + t.z);
        if (P & 2) {
          t = f3(s2.x + t.x, s2.y + t.y, s2.z + t.z);
          if (P & 4) t = f3(s3.x + t.x, s3.y + t.y, s3.z + t.z);
          else s3 = t;
        } else {
          s2 = t;
        }
      } else {
        s1 = t;
      }
      if (j + H == V) sum = t;  // the lane's sum
    }
    // the pixel's lanes pairwise: xor 1 and 2 by quad permutes (DPP), then
    // xor 4, 8, ... by shuffles
    F3 r = sum;
    r = f3(r.x + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(r.x), 0xB1, 0xf, 0xf, false)),
           r.y + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(r.y), 0xB1, 0xf, 0xf, false)),
           r.z + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(r.z), 0xB1, 0xf, 0xf, false)));
    r = f3(r.x + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(r.x), 0x4E, 0xf, 0xf, false)),
           r.y + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(r.y), 0x4E, 0xf, 0xf, false)),
           r.z + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(r.z), 0x4E, 0xf, 0xf, false)));
#pragma unroll
    for (int off = 4; off < LP; off <<= 1)
      r = f3(r.x + __shfl_xor(r.x, off), r.y + __shfl_xor(r.y, off), r.z + __shfl_xor(r.z, off));
    if (gg >= 0 && q == 0) {  // renderer.nim:159 (1 / samples.len), :204-209 (the pixel or its block)
      const F3 c = f3(r.x * p->inv_len, r.y * p->inv_len, r.z * p->inv_len);
      if (p->mode == 0 && p->step > 1) {
        const int xe = min(gp.x + p->step, p->width), ye = min(gp.y + p->step, p->height);
        for (int yy = gp.y; yy < ye; ++yy)
          for (int xx = gp.x; xx < xe; ++xx) {
            float* o = p->fb + ((size_t)yy * p->width + xx) * 3;
            o[0] = c.x; o[1] = c.y; o[2] = c.z;
          }
      } else {
        float* o = p->fb + ((size_t)gp.out_row * p->width + gp.x) * 3;
        o[0] = c.x; o[1] = c.y; o[2] = c.z;
      }
    }
    ws.v[STAT_PRIMARY] += pc(vmask) * (unsigned)V * (unsigned)iters;
    ws.v[STAT_SHADOW] += (unsigned)NL * nlit;
    ws.v[STAT_HITS] += nlit + nocc;
    if (++nflush >= p->stat_flush) {
      flush_stats(ws, tot, lane);
      nflush = 0;
    }
    g = wq.next();
  }
}

#ifndef RTMI_LEAN1Q_WAVES
#define RTMI_LEAN1Q_WAVES 8
#endif
template <int NL, int LP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RTMI_LEAN1Q_WAVES))) void k_render_lean1q(
    const FastParams params_by_value) {
  (void)params_by_value;
  const KP p = params();
  __shared__ unsigned long long lds_tot[4][kStatSlots];
  const int wib = (int)(threadIdx.x >> 6);
  const int lane = (int)__lane_id();
  if (lane < kStatSlots) lds_tot[wib][lane] = 0ull;
  Stats32 ws;
#pragma unroll
  for (int k = 0; k < kStatSlots; ++k) ws.v[k] = 0u;
  int nflush = 0;
  lean1q_loop<NL, LP>(p, p->order, list_items(p->list_n, p->ngroups, 64 / LP), p->queue, p->shards, ws,
                      lds_tot[wib], nflush);
  flush_stats(ws, lds_tot[wib], lane);
  const int wave = (int)(blockIdx.x * (blockDim.x >> 6) + threadIdx.x / 64u);
  if (lane < kStatSlots) p->partials[(size_t)wave * kStatSlots + lane] = lds_tot[wib][lane];
}

// The batched general-pixel kernel (two-class launches, rtmi.cpp
// split_lists): the launch's non-lean pixel groups (p->order lists them),
// each rendered by gen_batch from its pixel record, or — when a batch needs
// the BVH — by k_render_fast's one-sample loop (shade_path) from scratch.
// Used for scenes of one mesh object with distant lights only and no
// reflection (the subsets that have k_render_lean); frames and Stats
// bit-identical to k_render_fast.
#ifndef RTMI_GEN_BATCH
#define RTMI_GEN_BATCH 2
#endif
#ifndef RTMI_GEN_WAVES
#define RTMI_GEN_WAVES 7
#endif
constexpr int kGenBatch = RTMI_GEN_BATCH;
template <unsigned F>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(occ_table<F>(kOcc_gen, RTMI_GEN_WAVES)))) void
k_render_gen(
    const FastParams params_by_value) {
  (void)params_by_value;
  KP p = params();
  __shared__ float lds[4][kLdsSlots][64];  // gen_batch's albedo stash / shade_path's scratch (the fallback)
  extern __shared__ float sample_lds[];
  __shared__ unsigned long long lds_tot[4][kStatSlots];
  const int wib = (int)(threadIdx.x >> 6);
  LdsF* ls = (LdsF*)&lds[wib][0][__lane_id()];
  if (__lane_id() < (unsigned)kStatSlots) lds_tot[wib][__lane_id()] = 0ull;
  Stats32 ws;
#pragma unroll
  for (int k = 0; k < kStatSlots; ++k) ws.v[k] = 0u;
  const int shard = (int)(blockIdx.x % (unsigned int)p->shards);
  unsigned int* head = p->queue + shard * kQueueStride;
  int qj = 0;
  if (__lane_id() == 0) qj = (int)atomicAdd(head, 1u);
  qj = __builtin_amdgcn_readfirstlane(qj);
  int qj_next = 0;
  if (__lane_id() == 0) qj_next = (int)atomicAdd(head, 1u);
  int g = qj * p->shards + shard;
  int nflush = 0;
  const int ngroups = list_items(p->list_n, p->ngroups, 1);
  while (g < ngroups) {
    p = params();
    const int iters = p->iters;
    const int gg = cp(p->order)[g];
    GroupPix gp = group_pixel(p, gg, lane_id_fresh());
    gp.valid = true;  // the lists hold only pixels of the launch (rtmi.cpp split_lists)
    const LdsF* tb = sample_table<F>(p, gp, sample_lds, wib, 64);
    // the pixel's record (every listed group is one valid pixel)
    const unsigned pinfo = at(p->pix_info, __builtin_amdgcn_readfirstlane(gp.y * p->width + gp.x));
    Acc acc;
    acc.v = f3(0.0f, 0.0f, 0.0f);
    Stats32 wi;
#pragma unroll
    for (int k = 0; k < kStatSlots; ++k) wi.v[k] = 0u;
    // a pixel list past its slots (rt_frame.h): the one-sample loop, whose
    // camera rays take the BVH for this pixel
    bool ok = (pinfo & kPixCount) <= (1u << p->slot_lg);
    int it = 0;
    for (; ok && it + kGenBatch <= iters; it += kGenBatch) ok = gen_batch<F, kGenBatch>(p, gp, it, tb, pinfo, ls, acc, wi);
    for (; ok && it < iters; ++it) ok = gen_batch<F, 1>(p, gp, it, tb, pinfo, ls, acc, wi);
    if (params()->flags & RT_DEV_FLAG_FALLBACK) ok = false;  // test hook (RT_FLAG_BATCH_FALLBACK)
    if (ok) {
      ws.v[STAT_PRIMARY] += wi.v[STAT_PRIMARY];
      ws.v[STAT_SHADOW] += wi.v[STAT_SHADOW];
      ws.v[STAT_HITS] += wi.v[STAT_HITS];
#if defined(RTMI_DIAG_GEN_COUNT) || defined(RTMI_DIAG_LANES)
      for (int q = STAT_NODE_FETCH; q <= STAT_LANE_TRIS; ++q) ws.v[q] += wi.v[q];
#endif
    } else {  // some shadow ray needs the BVH: the whole pixel by the one-sample loop
      acc.v = f3(0.0f, 0.0f, 0.0f);
      ws.v[STAT_GEN_FALLBACK] += 1u;
      for (int i2 = 0; i2 < iters; ++i2) {
        p = params();
        const int s = i2 * 64 + gp.sub;
        const bool sv = gp.valid & (s < p->spp);
        const F3 d = camera_dir<F>(p, gp, s < p->spp ? s : 0, tb);
        const F3 o = f3(p->cam[0], p->cam[1], p->cam[2]);
        ws.v[STAT_PRIMARY] += pc(bal(sv));
        shade_path<false, F, false>(p, o, d, sv, sv ? gp.y * p->width + gp.x : -1, pinfo, ls, acc, ws);
      }
    }
    p = params();
    finish_item(p, gp, acc.v, 64);
    const int lane = lane_id_fresh();
    if (++nflush >= p->stat_flush) {
      flush_stats(ws, lds_tot[wib], lane);
      nflush = 0;
    }
    qj = __builtin_amdgcn_readfirstlane(qj_next);
    if (lane == 0) qj_next = (int)atomicAdd(head, 1u);
    g = qj * p->shards + shard;
  }
  p = params();
  const int lane = (int)__lane_id();
  flush_stats(ws, lds_tot[wib], lane);
  const int wave = (int)(blockIdx.x * (blockDim.x >> 6) + threadIdx.x / 64u);
  if (lane < kStatSlots) p->partials[(size_t)wave * kStatSlots + lane] = lds_tot[wib][lane];
}

// The batched general-pixel kernel of the one-plane scenes (rtmi.cpp
// one_plane_ok): k_render_gen with gen1_batch, NL distant lights.
#ifndef RTMI_GEN1_WAVES
#define RTMI_GEN1_WAVES 7
#endif
// k_render_gen1's work loop over the primary list (p->order, p->ngroups,
// the shard heads at p->queue); also the first phase of k_render_mix1.
template <int NL>
__device__ __forceinline__ void gen1_loop(KP p, LdsF* ls, Stats32& ws, unsigned long long* tot, int& nflush) {
  constexpr unsigned F = F_PLANE | F_MESH;
  WorkQ<RTMI_GEN_RUN> wq;
  int g = wq.start(p->queue, p->shards, list_items(p->list_n, p->ngroups, 1));
  while (g >= 0) {
    p = params();
    const int iters = p->iters;
    const int gg = cp(p->order)[g];
    GroupPix gp = group_pixel(p, gg, lane_id_fresh());
    gp.valid = true;  // the lists hold only pixels of the launch (rtmi.cpp split_lists)
    // a one-pixel group: its placement is wave-uniform (scalar registers;
    // per lane it stayed live as 64-bit products across the item and spilled)
    gp.x = __builtin_amdgcn_readfirstlane(gp.x);
    gp.y = __builtin_amdgcn_readfirstlane(gp.y);
    gp.out_row = __builtin_amdgcn_readfirstlane(gp.out_row);
    // the pixel index once per item, wave-uniform (recomputed per batch from
    // the lane's placement it kept a 64-bit product live and spilled)
    const int pu = __builtin_amdgcn_readfirstlane(gp.y * p->width + gp.x);
    const unsigned pinfo = at(p->pix_info, pu);
    Acc acc;
    acc.v = f3(0.0f, 0.0f, 0.0f);
    Stats32 wi;
#pragma unroll
    for (int k = 0; k < kStatSlots; ++k) wi.v[k] = 0u;
    // a pixel list past its slots (rt_frame.h): the one-sample loop, whose
    // camera rays take the BVH for this pixel
    bool ok = (pinfo & kPixCount) <= (1u << p->slot_lg);
    for (int it = 0; ok && it < iters; it += kGenBatch) ok = gen1_batch<kGenBatch, NL>(p, gp, pu, it, pinfo, acc, wi);
    if (params()->flags & RT_DEV_FLAG_FALLBACK) ok = false;  // test hook (RT_FLAG_BATCH_FALLBACK)
    if (ok) {
      ws.v[STAT_PRIMARY] += wi.v[STAT_PRIMARY];
      ws.v[STAT_SHADOW] += wi.v[STAT_SHADOW];
      ws.v[STAT_HITS] += wi.v[STAT_HITS];
#if defined(RTMI_DIAG_GEN_COUNT) || defined(RTMI_DIAG_LANES)
      for (int q = STAT_NODE_FETCH; q <= STAT_LANE_TRIS; ++q) ws.v[q] += wi.v[q];
#endif
    } else {  // some shadow ray needs the BVH: the whole pixel by the one-sample loop
      acc.v = f3(0.0f, 0.0f, 0.0f);
      ws.v[STAT_GEN_FALLBACK] += 1u;
      for (int i2 = 0; i2 < iters; ++i2) {
        p = params();
        const int s = i2 * 64 + gp.sub;
        const F3 d = camera_dir<F>(p, gp, s, nullptr);
        const F3 o = f3(p->cam[0], p->cam[1], p->cam[2]);
        ws.v[STAT_PRIMARY] += 64u;
        shade_path<false, F, false>(p, o, d, true, gp.y * p->width + gp.x, pinfo, ls, acc, ws);
      }
    }
    p = params();
    finish_item(p, gp, acc.v, 64);
    const int lane = lane_id_fresh();
    if (++nflush >= p->stat_flush) {
      flush_stats(ws, tot, lane);
      nflush = 0;
    }
    g = wq.next();
  }
}

template <int NL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RTMI_GEN1_WAVES))) void k_render_gen1(
    const FastParams params_by_value) {
  (void)params_by_value;
  KP p = params();
  __shared__ float lds[4][kLdsSlots][64];  // shade_path's scratch (the fallback)
  __shared__ unsigned long long lds_tot[4][kStatSlots];
  // the wave's index in its block as a scalar (from threadIdx.x it stayed a
  // VGPR live across the whole item loop and spilled, as did the LDS address
  // of lds_tot[wib] formed from it)
  const int wib = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  LdsF* ls = (LdsF*)&lds[wib][0][__lane_id()];
  if (__lane_id() < (unsigned)kStatSlots) lds_tot[wib][__lane_id()] = 0ull;
  Stats32 ws;
#pragma unroll
  for (int k = 0; k < kStatSlots; ++k) ws.v[k] = 0u;
  int nflush = 0;
  gen1_loop<NL>(p, ls, ws, lds_tot[wib], nflush);
  p = params();
  const int lane = (int)__lane_id();
  flush_stats(ws, lds_tot[wib], lane);
  const int wave = (int)(blockIdx.x * 4u) + wib;  // (256-thread blocks)
  if (lane < kStatSlots) p->partials[(size_t)wave * kStatSlots + lane] = lds_tot[wib][lane];
}

// Both classes of a one-plane two-class launch in ONE kernel (short
// launches, rtmi.cpp): every wave takes general pixels (k_render_gen1's
// items, p->order / p->ngroups) until that list is exhausted, then lean
// pixels (k_render_lean1q's items, p->order2 / p->ngroups2 from the second
// set of queue heads) — one ramp and one tail per launch instead of two, the
// expensive items first and the cheap ones filling the tail. Frames and
// Stats those of the two kernels.
template <int NL, int LP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RTMI_GEN1_WAVES))) void k_render_mix1(
    const FastParams params_by_value) {
  (void)params_by_value;
  KP p = params();
  __shared__ float lds[4][kLdsSlots][64];
  __shared__ unsigned long long lds_tot[4][kStatSlots];
  // the wave's index in its block as a scalar (from threadIdx.x it stayed a
  // VGPR live across the whole item loop and spilled, as did the LDS address
  // of lds_tot[wib] formed from it)
  const int wib = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  LdsF* ls = (LdsF*)&lds[wib][0][__lane_id()];
  if (__lane_id() < (unsigned)kStatSlots) lds_tot[wib][__lane_id()] = 0ull;
  Stats32 ws;
#pragma unroll
  for (int k = 0; k < kStatSlots; ++k) ws.v[k] = 0u;
  int nflush = 0;
  gen1_loop<NL>(p, ls, ws, lds_tot[wib], nflush);
  p = params();
  lean1q_loop<NL, LP>(p, p->order2, list_items(p->list_n2, p->ngroups2, 64 / LP), p->queue + kQueueShards * kQueueStride, p->shards2, ws,
                      lds_tot[wib], nflush);
  p = params();
  const int lane = (int)__lane_id();
  flush_stats(ws, lds_tot[wib], lane);
  const int wave = (int)(blockIdx.x * 4u) + wib;  // (256-thread blocks)
  if (lane < kStatSlots) p->partials[(size_t)wave * kStatSlots + lane] = lds_tot[wib][lane];
}

}  // namespace fast
}  // namespace rtmi
