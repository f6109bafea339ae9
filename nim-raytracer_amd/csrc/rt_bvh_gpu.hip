// rt_bvh_gpu.hip — device BVH2 builder (rt_scene_desc.bvh_builder =
// RT_BVH_PLOC): the same node format, leaf rule and conservative float32
// bounds as the host binned-SAH builder (rt_bvh.cpp), built on the GPU.
//
//   1. face bounds (float64) reduced to the mesh bounds -> the margin the host
//      builder uses (2^-20 of the mesh scale); per face: float64 box inflated
//      by it and rounded outward to float32, 63-bit Morton code of its centre
//   2. rocPRIM radix sort of (code, face)
//   3. PLOC (parallel locally-ordered clustering): every cluster finds the
//      neighbour within +-16 sorted positions whose merged box has the least
//      area; mutual pairs merge; an exclusive scan compacts the survivors and
//      numbers the new nodes. Repeats until one cluster is left. Ties go to
//      the lower position, so the globally closest pair is always mutual and
//      every round merges at least one pair.
//   4. bottom-up SAH pass (second arrival at a node continues): a subtree of
//      <= max_leaf faces becomes one leaf when n * C_tri <= its split cost
//   5. layout by walking up from every node: a leaf's first face slot and an
//      inner node's index are sums over its ancestors, which gives the host
//      builder's depth-first (left first) order without a sequential pass
//
// The reference has no acceleration structure (TriangleMesh.intersect,
// src/renderer/geom.nim:339-358, loops over every face); like the host
// builder's, these bounds make traversal return the brute-force answer, so
// images and Stats do not depend on which builder made the tree.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rt_bvh.h"

namespace rtmi {
namespace {

constexpr int kRadius = 32;  // largest PLOC neighbourhood (sorted positions each side)
constexpr int kBlock = 256;
constexpr int kMortonBits = 21;

struct Box32 {
  float lo[3], hi[3];
};

__device__ __forceinline__ unsigned long long ord_bits(double x) {  // monotone double -> u64
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

double unord_bits(unsigned long long k) {
  const unsigned long long b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  double x;
  std::memcpy(&x, &b, sizeof x);
  return x;
}

__device__ __forceinline__ float half_area(const Box32& b) {
  const float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
  return dx * dy + dy * dz + dz * dx;
}

__device__ __forceinline__ Box32 unite(const Box32& a, const Box32& b) {
  Box32 r;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    r.lo[k] = fminf(a.lo[k], b.lo[k]);
    r.hi[k] = fmaxf(a.hi[k], b.hi[k]);
  }
  return r;
}

__device__ __forceinline__ unsigned long long spread21(unsigned long long x) {
  x &= 0x1fffffull;
  x = (x | x << 32) & 0x1f00000000ffffull;
  x = (x | x << 16) & 0x1f0000ff0000ffull;
  x = (x | x << 8) & 0x100f00f00f00f00full;
  x = (x | x << 4) & 0x10c30c30c30c30c3ull;
  x = (x | x << 2) & 0x1249249249249249ull;
  return x;
}

// 1a. mesh bounds over the faces' vertices (6 ordered-bit words: lo xyz, hi xyz)
__global__ __launch_bounds__(kBlock) void k_bounds(const double* v, const int32_t* f, long long nf,
                                                    unsigned long long* out) {
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (long long t = (long long)blockIdx.x * kBlock + threadIdx.x; t < nf; t += (long long)gridDim.x * kBlock)
    for (int k = 0; k < 3; ++k) {
      const double* p = v + 3 * (size_t)f[3 * t + k];
      for (int a = 0; a < 3; ++a) {
        lo[a] = fmin(lo[a], p[a]);
        hi[a] = fmax(hi[a], p[a]);
      }
    }
  __shared__ double s[6][kBlock];
  for (int a = 0; a < 3; ++a) {
    s[a][threadIdx.x] = lo[a];
    s[3 + a][threadIdx.x] = hi[a];
  }
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int a = 0; a < 3; ++a) {
        s[a][threadIdx.x] = fmin(s[a][threadIdx.x], s[a][threadIdx.x + w]);
        s[3 + a][threadIdx.x] = fmax(s[3 + a][threadIdx.x], s[3 + a][threadIdx.x + w]);
      }
    __syncthreads();
  }
  if (threadIdx.x == 0)
    for (int a = 0; a < 3; ++a) {
      atomicMin(&out[a], ord_bits(s[a][0]));
      atomicMax(&out[3 + a], ord_bits(s[3 + a][0]));
    }
}

struct LeafArgs {
  double inflate;
  double lo[3], scale[3];  // Morton quantisation of face centres
};

// 1b. per face: conservative float32 box (rt_bvh.cpp lo32/hi32) + Morton code
__global__ __launch_bounds__(kBlock) void k_leaves(const double* v, const int32_t* f, long long nf, LeafArgs a,
                                                    Box32* box, unsigned long long* key, int32_t* id) {
  const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (t >= nf) return;
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int k = 0; k < 3; ++k) {
    const double* p = v + 3 * (size_t)f[3 * t + k];
    for (int c = 0; c < 3; ++c) {
      lo[c] = fmin(lo[c], p[c]);
      hi[c] = fmax(hi[c], p[c]);
    }
  }
  Box32 b;
  unsigned long long code = 0;
  for (int c = 0; c < 3; ++c) {
    b.lo[c] = __double2float_rd(lo[c] - a.inflate);
    b.hi[c] = __double2float_ru(hi[c] + a.inflate);
    const double q = (0.5 * (lo[c] + hi[c]) - a.lo[c]) * a.scale[c];
    const unsigned long long qi =
        (unsigned long long)fmin(fmax(q, 0.0), (double)((1u << kMortonBits) - 1));
    code |= spread21(qi) << (2 - c);
  }
  box[t] = b;
  key[t] = code;
  id[t] = (int32_t)t;
}

__global__ __launch_bounds__(kBlock) void k_init(const int32_t* sorted, int n, const Box32* box, int32_t* cl_id,
                                                  Box32* cl_box) {
  const int i = (int)(blockIdx.x * kBlock + threadIdx.x);
  if (i >= n) return;
  const int32_t t = sorted[i];
  cl_id[i] = t;
  cl_box[i] = box[t];
}

__device__ __forceinline__ unsigned pair_hash(unsigned lo, unsigned hi) {
  unsigned h = lo * 0x9E3779B1u ^ (hi + 0x7F4A7C15u) * 0x85EBCA77u;
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  h ^= h >> 15;
  h *= 0x846CA68Bu;
  h ^= h >> 16;
  return h;
}

// 3a. nearest neighbour by merged-box area within +-kRadius sorted positions.
// A pair's distance is (area, hash of the pair, lower position, higher
// position), compared lexicographically: symmetric and never tied, so the
// globally closest pair is always mutual (every round merges). The hash
// decides between equal areas at random instead of by position — with
// position as the tie-break, coincident faces (all merged areas equal) pair
// up one per round into a chain as deep as their count.
__global__ __launch_bounds__(kBlock) void k_nearest(const Box32* cl_box, int n, int radius, int32_t* nn) {
  __shared__ Box32 sb[kBlock + 2 * kRadius];
  const int base = (int)blockIdx.x * kBlock;
  for (int k = (int)threadIdx.x; k < kBlock + 2 * kRadius; k += kBlock) {
    const int j = base - kRadius + k;
    if (j >= 0 && j < n) sb[k] = cl_box[j];
  }
  __syncthreads();
  const int i = base + (int)threadIdx.x;
  if (i >= n) return;
  const Box32 bi = sb[threadIdx.x + kRadius];
  unsigned long long best = ~0ull;
  int bj = -1;
  for (int d = -radius; d <= radius; ++d) {
    const int j = i + d;
    if (d == 0 || j < 0 || j >= n) continue;
    const float s = half_area(unite(bi, sb[(int)threadIdx.x + kRadius + d]));
    const unsigned lo = (unsigned)min(i, j), hi = (unsigned)max(i, j);
    // areas are >= 0, so their bit patterns order like the values
    const unsigned long long key = ((unsigned long long)__float_as_uint(s) << 32) | pair_hash(lo, hi);
    if (key < best || (key == best && j < bj)) {  // equal key: the lower position (ties are then
      best = key;                                  // decided by position, consistently on both sides)
      bj = j;
    }
  }
  nn[i] = bj;
}

// 3b. survivors (bit 0) and merge owners (bit 32) for one exclusive scan
__global__ __launch_bounds__(kBlock) void k_flags(const int32_t* nn, int n, unsigned long long* flags) {
  const int i = (int)(blockIdx.x * kBlock + threadIdx.x);
  if (i >= n) return;
  const int j = nn[i];
  const bool mutual = nn[j] == i;
  flags[i] = (mutual && i > j ? 0ull : 1ull) | ((mutual && i < j) ? (1ull << 32) : 0ull);
}

// 3c. compaction + node creation (node = first_node + merge rank: deterministic)
__global__ __launch_bounds__(kBlock) void k_merge(int n, const int32_t* nn, const unsigned long long* flags,
                                                   const unsigned long long* pos, const int32_t* cl_id,
                                                   const Box32* cl_box, int32_t* out_id, Box32* out_box,
                                                   int32_t nf, int32_t first_node, int2* children, Box32* node_box,
                                                   int32_t* parent) {
  const int i = (int)(blockIdx.x * kBlock + threadIdx.x);
  if (i >= n) return;
  const unsigned long long fl = flags[i];
  if (!(fl & 1ull)) return;
  const int o = (int)(pos[i] & 0xffffffffull);
  if (fl >> 32) {
    const int j = nn[i];
    const int32_t node = first_node + (int32_t)(pos[i] >> 32);
    const int32_t a = cl_id[i], b = cl_id[j];
    const Box32 u = unite(cl_box[i], cl_box[j]);
    children[node - nf] = make_int2(a, b);
    node_box[node] = u;
    parent[a] = node;
    parent[b] = node;
    out_id[o] = node;
    out_box[o] = u;
  } else {
    out_id[o] = cl_id[i];
    out_box[o] = cl_box[i];
  }
}

__global__ void k_total(const unsigned long long* pos, const unsigned long long* flags, int n,
                        unsigned long long* tot) {
  tot[0] = pos[n - 1] + flags[n - 1];
}

struct NodeInfo {  // bottom-up results per node (faces, SAH cost, leaf?, inner nodes kept)
  int32_t nfaces;
  float cost;
  int32_t leaf;
  int32_t inner;
};

// 4. bottom-up SAH: the second thread to reach a node evaluates it
__global__ __launch_bounds__(kBlock) void k_collapse(int32_t nf, const int32_t* parent, const int2* children,
                                                      const Box32* node_box, int32_t* visits, NodeInfo* info,
                                                      int max_leaf, float c_node, float c_tri) {
  const int32_t t = (int32_t)(blockIdx.x * kBlock + threadIdx.x);
  if (t >= nf) return;
  volatile NodeInfo* vi = info;
  vi[t].nfaces = 1;
  vi[t].cost = c_tri;
  vi[t].leaf = 1;
  vi[t].inner = 0;
  int32_t v = t;
  for (;;) {
    const int32_t p = parent[v];
    if (p < 0) break;
    __threadfence();
    if (atomicAdd(&visits[p - nf], 1) == 0) return;
    __threadfence();
    const int2 ch = children[p - nf];
    const int32_t n = vi[ch.x].nfaces + vi[ch.y].nfaces;
    const float A = half_area(node_box[p]);
    const float sl = half_area(node_box[ch.x]), sr = half_area(node_box[ch.y]);
    const float cl = vi[ch.x].cost, cr = vi[ch.y].cost;
    const float split = c_node + (A > 0.0f ? (sl * cl + sr * cr) / A : 0.5f * (cl + cr));
    // (pricing the children as leaves, like rt_bvh.cpp, changed 0.1 % of
    // the nodes and nothing measurable)
    const bool leaf = n <= max_leaf && (float)n * c_tri <= split;
    vi[p].nfaces = n;
    vi[p].cost = leaf ? (float)n * c_tri : split;
    vi[p].leaf = leaf ? 1 : 0;
    vi[p].inner = leaf ? 0 : 1 + vi[ch.x].inner + vi[ch.y].inner;
    v = p;
  }
}

// 5a. every kept node walks to the root: a leaf sums its left-sibling face
// counts (first face slot) and lists its faces depth-first; an inner node
// sums 1 + left-sibling inner counts (its depth-first index)
__global__ __launch_bounds__(kBlock) void k_layout(int32_t nf, int32_t nnodes, const int32_t* parent,
                                                    const int2* children, const NodeInfo* info, int max_leaf,
                                                    int32_t* slot, int32_t* index, int32_t* order,
                                                    int32_t* depth_max) {
  const int32_t v = (int32_t)(blockIdx.x * kBlock + threadIdx.x);
  if (v >= nnodes) return;
  for (int32_t u = v;;) {  // inside a collapsed subtree? (only ancestors with <= max_leaf faces can be)
    const int32_t p = parent[u];
    if (p < 0 || info[p].nfaces > max_leaf) break;
    if (info[p].leaf) return;
    u = p;
  }
  if (info[v].leaf) {
    int32_t off = 0;
    for (int32_t u = v, p; (p = parent[u]) >= 0; u = p) {
      const int2 ch = children[p - nf];
      if (ch.y == u) off += info[ch.x].nfaces;
    }
    slot[v] = off;
    int32_t stack[2 * kLeafMax + 2];
    int sp = 0, k = 0;
    stack[sp++] = v;
    while (sp > 0) {
      const int32_t w = stack[--sp];
      if (w < nf) {
        order[off + k++] = w;
      } else {
        const int2 ch = children[w - nf];
        stack[sp++] = ch.y;
        stack[sp++] = ch.x;
      }
    }
  } else {
    int32_t id = 0, depth = 1;
    for (int32_t u = v, p; (p = parent[u]) >= 0; u = p, ++depth) {
      const int2 ch = children[p - nf];
      id += 1 + (ch.y == u ? info[ch.x].inner : 0);
    }
    index[v] = id;
    atomicMax(depth_max, depth);
  }
}

// 5b. one BvhNode per kept inner node
__global__ __launch_bounds__(kBlock) void k_emit(int32_t nf, int32_t ninner, const int2* children,
                                                  const NodeInfo* info, const Box32* node_box, const int32_t* slot,
                                                  const int32_t* index, BvhNode* out) {
  const int32_t p = nf + (int32_t)(blockIdx.x * kBlock + threadIdx.x);
  if (p - nf >= ninner) return;
  const int32_t me = index[p];
  if (me < 0 || info[p].leaf) return;
  const int2 ch = children[p - nf];
  BvhNode nd;
  const int32_t cs[2] = {ch.x, ch.y};
  for (int k = 0; k < 2; ++k) {
    const int32_t c = cs[k];
    const Box32 b = node_box[c];
    float* lo = k == 0 ? nd.lo0 : nd.lo1;
    float* hi = k == 0 ? nd.hi0 : nd.hi1;
    for (int a = 0; a < 3; ++a) {
      lo[a] = b.lo[a];
      hi[a] = b.hi[a];
    }
    const int32_t cref = info[c].leaf ? slot[c] : index[c];
    const int32_t cn = info[c].leaf ? info[c].nfaces : 0;
    if (k == 0) {
      nd.c0 = cref;
      nd.n0 = cn;
    } else {
      nd.c1 = cref;
      nd.n1 = cn;
    }
  }
  out[me] = nd;
}

template <class T>
struct Dev {
  T* p = nullptr;
  ~Dev() {
    if (p) (void)hipFree(p);
  }
  bool alloc(size_t n) { return hipMalloc((void**)&p, std::max<size_t>(n, 1) * sizeof(T)) == hipSuccess; }
};

unsigned grid(long long n) { return (unsigned)((n + kBlock - 1) / kBlock); }


// Triangle records in leaf order. Edges and the cross product in float64
// (-ffp-contract=off, as rtmi.cpp's host code), rounded to float32 once.
__global__ __launch_bounds__(kBlock) void k_pack(const double* v, const int32_t* f, const int32_t* order,
                                                  long long nf, TriFast* fast, TriF64* f64) {
  const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (i >= nf) return;
  const int32_t face = order[i];
  const int32_t* fi = f + 3 * (size_t)face;
  const double* v0 = v + 3 * (size_t)fi[0];
  const double* v1 = v + 3 * (size_t)fi[1];
  const double* v2 = v + 3 * (size_t)fi[2];
  double e1[3], e2[3];
  for (int k = 0; k < 3; ++k) {
    e1[k] = v1[k] - v0[k];  // v0v1 exactly as geom.nim:286-288
    e2[k] = v2[k] - v0[k];  // v0v2 exactly as geom.nim:292-294
  }
  const double n[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                       e1[0] * e2[1] - e1[1] * e2[0]};
  TriFast t;
  TriF64 d;
  for (int k = 0; k < 3; ++k) {
    t.v0[k] = (float)v0[k];
    t.e2[k] = (float)e2[k];
    t.e1n[k] = (float)-e1[k];
    t.nn[k] = (float)-n[k];
    d.v0[k] = v0[k];
    d.e1[k] = e1[k];
    d.e2[k] = e2[k];
  }
  t.id = face;
  t.pad0 = t.pad1 = t.pad2 = 0.0f;
  d.id = face;
  d.pad = 0;
  fast[i] = t;
  f64[i] = d;
}

}  // namespace

bool pack_triangles_device(const double* d_v, const int32_t* d_f, const int32_t* d_order, int64_t nf,
                           TriFast* d_fast, TriF64* d_f64, void* stream) {
  if (nf <= 0) return true;
  k_pack<<<grid(nf), kBlock, 0, (hipStream_t)stream>>>(d_v, d_f, d_order, nf, d_fast, d_f64);
  return hipGetLastError() == hipSuccess;
}

bool build_bvh_device(const double* d_vin, const int32_t* d_fin, int64_t nf, const BvhBuildParams& prm,
                      BvhResult* out, const char** err) {
  out->nodes.clear();
  out->order.clear();
  out->max_depth = 0;
  if (nf <= 0) return true;
  if (nf > ((int64_t)1 << 29)) {
    *err = "mesh too large for the device builder (> 2^29 faces)";
    return false;
  }
  const int32_t n = (int32_t)nf;
  const int32_t nnodes = 2 * n - 1;
  hipStream_t st = nullptr;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
    *err = "device BVH build: stream creation failed";
    return false;
  }
  struct StreamGuard {
    hipStream_t s;
    ~StreamGuard() { (void)hipStreamDestroy(s); }
  } sg{st};
#define DEV_OK(expr)                                  \
  do {                                                \
    if ((expr) != hipSuccess) {                       \
      *err = "device BVH build: " #expr " failed";    \
      return false;                                   \
    }                                                 \
  } while (0)

  const double* d_v = d_vin;
  const int32_t* d_f = d_fin;
  Dev<unsigned long long> d_bounds, d_key, d_key2, d_flags, d_pos, d_tot;
  Dev<Box32> d_box, d_cl_box[2];
  Dev<int32_t> d_id, d_id2, d_cl_id[2], d_nn, d_parent, d_visits, d_slot, d_index, d_order, d_depth;
  Dev<int2> d_children;
  Dev<Box32> d_node_box;
  Dev<NodeInfo> d_info;
  if (!d_bounds.alloc(6) || !d_key.alloc(n) ||
      !d_key2.alloc(n) || !d_flags.alloc(n) || !d_pos.alloc(n) || !d_tot.alloc(1) || !d_box.alloc(n) ||
      !d_cl_box[0].alloc(n) || !d_cl_box[1].alloc(n) || !d_id.alloc(n) || !d_id2.alloc(n) ||
      !d_cl_id[0].alloc(n) || !d_cl_id[1].alloc(n) || !d_nn.alloc(n) || !d_parent.alloc(nnodes) ||
      !d_visits.alloc(n) || !d_slot.alloc(nnodes) || !d_index.alloc(nnodes) || !d_order.alloc(n) ||
      !d_depth.alloc(1) || !d_children.alloc(n) || !d_node_box.alloc(nnodes) || !d_info.alloc(nnodes)) {
    *err = "device BVH build: out of device memory";
    return false;
  }

  // 1. mesh bounds -> margin and Morton frame
  unsigned long long init[6];
  for (int a = 0; a < 3; ++a) {
    init[a] = ~0ull;
    init[3 + a] = 0ull;
  }
  DEV_OK(hipMemcpyAsync(d_bounds.p, init, sizeof init, hipMemcpyHostToDevice, st));
  k_bounds<<<std::min(grid(n), 2048u), kBlock, 0, st>>>(d_v, d_f, n, d_bounds.p);
  unsigned long long hb[6];
  DEV_OK(hipMemcpyAsync(hb, d_bounds.p, sizeof hb, hipMemcpyDeviceToHost, st));
  DEV_OK(hipStreamSynchronize(st));
  double lo[3], hi[3], mag = 0.0, extent = 0.0;
  for (int a = 0; a < 3; ++a) {
    lo[a] = unord_bits(hb[a]);
    hi[a] = unord_bits(hb[3 + a]);
    mag = std::max(mag, std::max(std::fabs(lo[a]), std::fabs(hi[a])));
    extent = std::max(extent, hi[a] - lo[a]);
  }
  if (!std::isfinite(mag) || !std::isfinite(extent)) {
    *err = "mesh has non-finite vertices";
    return false;
  }
  LeafArgs la;
  la.inflate = std::ldexp(std::max(extent, mag), -20) + 1e-30;  // = rt_bvh.cpp
  for (int a = 0; a < 3; ++a) {
    la.lo[a] = lo[a];
    const double e = hi[a] - lo[a];
    la.scale[a] = e > 0.0 ? (double)(1u << kMortonBits) / e : 0.0;
  }
  k_leaves<<<grid(n), kBlock, 0, st>>>(d_v, d_f, n, la, d_box.p, d_key.p, d_id.p);

  // 2. Morton order
  size_t sort_bytes = 0, scan_bytes = 0;
  DEV_OK(rocprim::radix_sort_pairs(nullptr, sort_bytes, d_key.p, d_key2.p, d_id.p, d_id2.p, n, 0, 3 * kMortonBits,
                                   st));
  DEV_OK(rocprim::exclusive_scan(nullptr, scan_bytes, d_flags.p, d_pos.p, 0ull, (size_t)n,
                                 rocprim::plus<unsigned long long>(), st));
  Dev<unsigned char> d_tmp;
  if (!d_tmp.alloc(std::max(sort_bytes, scan_bytes))) {
    *err = "device BVH build: out of device memory";
    return false;
  }
  DEV_OK(rocprim::radix_sort_pairs(d_tmp.p, sort_bytes, d_key.p, d_key2.p, d_id.p, d_id2.p, n, 0, 3 * kMortonBits,
                                   st));
  k_init<<<grid(n), kBlock, 0, st>>>(d_id2.p, n, d_box.p, d_cl_id[0].p, d_cl_box[0].p);
  DEV_OK(hipMemcpyAsync(d_node_box.p, d_box.p, (size_t)n * sizeof(Box32), hipMemcpyDeviceToDevice, st));
  DEV_OK(hipMemsetAsync(d_parent.p, 0xff, (size_t)nnodes * sizeof(int32_t), st));

  // search radius: 16 (8 and 32 traced no faster: C3 8.53 / 8.57 ms vs
  // 8.24, 1M-face torus 3.84 / 3.94 vs 3.84); RTMI_PLOC_RADIUS overrides
  static const int radius = [] {
    const char* e = rtmi::diag_env("RTMI_PLOC_RADIUS");
    return e ? std::max(1, std::min(kRadius, std::atoi(e))) : 16;
  }();
  // 3. PLOC rounds: every round merges at least the globally closest pair
  int cur = 0, live = n;
  int32_t next_node = n;
  for (int round = 0; live > 1; ++round) {
    if (round > n) {
      *err = "device BVH build: clustering made no progress";
      return false;
    }
    k_nearest<<<grid(live), kBlock, 0, st>>>(d_cl_box[cur].p, live, radius, d_nn.p);
    k_flags<<<grid(live), kBlock, 0, st>>>(d_nn.p, live, d_flags.p);
    size_t bytes = scan_bytes;
    DEV_OK(rocprim::exclusive_scan(d_tmp.p, bytes, d_flags.p, d_pos.p, 0ull, (size_t)live,
                                   rocprim::plus<unsigned long long>(), st));
    k_merge<<<grid(live), kBlock, 0, st>>>(live, d_nn.p, d_flags.p, d_pos.p, d_cl_id[cur].p, d_cl_box[cur].p,
                                           d_cl_id[cur ^ 1].p, d_cl_box[cur ^ 1].p, n, next_node, d_children.p,
                                           d_node_box.p, d_parent.p);
    k_total<<<1, 1, 0, st>>>(d_pos.p, d_flags.p, live, d_tot.p);
    unsigned long long tot = 0;
    DEV_OK(hipMemcpyAsync(&tot, d_tot.p, sizeof tot, hipMemcpyDeviceToHost, st));
    DEV_OK(hipStreamSynchronize(st));
    const int survivors = (int)(tot & 0xffffffffull), merged = (int)(tot >> 32);
    if (merged <= 0 || survivors != live - merged) {
      *err = "device BVH build: clustering made no progress";
      return false;
    }
    next_node += merged;
    live = survivors;
    cur ^= 1;
  }
  if (next_node != nnodes) {
    *err = "device BVH build: wrong node count";
    return false;
  }
  int32_t root = 0;
  DEV_OK(hipMemcpyAsync(&root, d_cl_id[cur].p, sizeof root, hipMemcpyDeviceToHost, st));

  // 4. SAH collapse into leaves of <= max_leaf faces
  DEV_OK(hipMemsetAsync(d_visits.p, 0, (size_t)n * sizeof(int32_t), st));
  k_collapse<<<grid(n), kBlock, 0, st>>>(n, d_parent.p, d_children.p, d_node_box.p, d_visits.p, d_info.p,
                                         prm.max_leaf, prm.cost_node, prm.cost_tri);
  NodeInfo ri;
  DEV_OK(hipMemcpyAsync(&ri, d_info.p + root, sizeof ri, hipMemcpyDeviceToHost, st));
  DEV_OK(hipStreamSynchronize(st));
  if (ri.nfaces != n) {
    *err = "device BVH build: tree does not cover every face";
    return false;
  }

  // 5. depth-first layout
  DEV_OK(hipMemsetAsync(d_index.p, 0xff, (size_t)nnodes * sizeof(int32_t), st));
  DEV_OK(hipMemsetAsync(d_depth.p, 0, sizeof(int32_t), st));
  k_layout<<<grid(nnodes), kBlock, 0, st>>>(n, nnodes, d_parent.p, d_children.p, d_info.p, prm.max_leaf, d_slot.p,
                                            d_index.p, d_order.p, d_depth.p);
  const int32_t ninner = ri.leaf ? 0 : ri.inner;
  Dev<BvhNode> d_out;
  if (!d_out.alloc(std::max(ninner, 1))) {
    *err = "device BVH build: out of device memory";
    return false;
  }
  if (ninner > 0)
    k_emit<<<grid(n - 1), kBlock, 0, st>>>(n, n - 1, d_children.p, d_info.p, d_node_box.p, d_slot.p, d_index.p,
                                           d_out.p);
  out->order.resize((size_t)n);
  DEV_OK(hipMemcpyAsync(out->order.data(), d_order.p, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
  int32_t depth = 0;
  DEV_OK(hipMemcpyAsync(&depth, d_depth.p, sizeof depth, hipMemcpyDeviceToHost, st));
  if (ninner > 0) {
    out->nodes.resize((size_t)ninner);
    DEV_OK(hipMemcpyAsync(out->nodes.data(), d_out.p, (size_t)ninner * sizeof(BvhNode), hipMemcpyDeviceToHost, st));
  } else {  // the whole mesh is one leaf: the root repeats it in both slots (rt_bvh.cpp)
    Box32 rb;
    DEV_OK(hipMemcpyAsync(&rb, d_node_box.p + root, sizeof rb, hipMemcpyDeviceToHost, st));
    DEV_OK(hipStreamSynchronize(st));
    BvhNode nd;
    for (int a = 0; a < 3; ++a) {
      nd.lo0[a] = nd.lo1[a] = rb.lo[a];
      nd.hi0[a] = nd.hi1[a] = rb.hi[a];
    }
    nd.c0 = nd.c1 = 0;
    nd.n0 = nd.n1 = n;
    out->nodes.push_back(nd);
    depth = 1;
  }
  DEV_OK(hipStreamSynchronize(st));
#undef DEV_OK
  out->max_depth = std::max(1, depth);
  if (out->max_depth > kMaxBvhDepth) {
    *err = "BVH deeper than the traversal stack";
    return false;
  }
  return validate_bvh(*out, nf, err);
}

}  // namespace rtmi
