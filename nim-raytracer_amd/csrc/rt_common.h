// rt_common.h — device-resident scene layout shared by the host library
// (rtmi.cpp) and the gfx950 kernels (rt_device.h).
//
// HBM layout (all arrays resident for the scene's lifetime, built once by
// rt_scene_create):
//   objects  DevObject<R>[nobj]   scene order (trace order, renderer.nim:53)
//   lights   DevLight<R>[nlight]
//   meshes   DevMesh<R>[nmesh]
//   nodes    BvhNode[...]         64-B BVH2 nodes, both child boxes per node,
//                                 depth-first order, all meshes concatenated
//   tris     TriRec<R>[...]       leaf-ordered triangles (v0, e1, e2, face id)
//   normals  R[3 * faces]         one face normal per ORIGINAL face index
//                                 (obj.nim calcNormals), looked up by face id
#pragma once
#include <stdint.h>
#include <stdlib.h>

namespace rtmi {

// Diagnostic and A/B knobs (RTMI_* environment variables: launch shapes,
// occupancy caps, probe modes that give wrong images on purpose) are read
// only by libraries built with -DRTMI_DIAG (tools/build_variant.sh); the
// production library ignores them.
inline const char* diag_env(const char* name) {
#ifdef RTMI_DIAG
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

enum : int32_t { GEOM_SPHERE = 0, GEOM_PLANE = 1, GEOM_BOX = 2, GEOM_MESH = 3 };
enum : int32_t { LIGHT_DISTANT = 0, LIGHT_POINT = 1 };
// DevObject.xf: what world_to_object is (host-classified, float32 fast paths)
enum : int32_t { XF_IDENTITY = 0, XF_TRANSLATE = 1, XF_GENERAL = 2 };
// RenderParams.flags bits
enum : int32_t { RT_DEV_FLAG_COUNT = 0x2, RT_DEV_FLAG_FALLBACK = 0x40, RT_DEV_FLAG_NO_OBJ_BATCH = 0x1000 };

constexpr int kMaxBvhDepth = 60;      // stack fits one 64-lane VGPR
constexpr int kLeafMax = 4;           // triangles per BVH leaf (arrays padded by kLeafMax-1)
constexpr int kMaxShadeLevels = 8;    // primary + 7 reflection bounces
constexpr int kStatSlots = 10;        // per-wave partial counters

// Geometry + material record. Matrices column-major like glm.
template <class R>
struct alignas(16) DevObject {
  R w2o[16];
  R o2w[16];
  R prm[8];      // sphere: prm[0] = r; box: prm[0..2] = vmin, prm[4..6] = vmax
  R albedo[4];   // rgb, reflection
  R albp[4];     // albedo / PI (rgb), formed by the host in R: the IEEE quotient
                 // shadeDiffuse's `albedo / PI` gives (shader.nim:15), read by
                 // the float64 kernels instead of dividing per sample
  int32_t type;
  int32_t mesh;
  int32_t xf;          // XF_* classification of world_to_object
  int32_t pad1;
};

template <class R>
struct alignas(16) DevLight {
  R ci[4];       // color * intensity (rgb)  (light.nim:50,57)
  R v[4];        // distant: dir; point: pos
  int32_t type;
  int32_t pad[3];
};

template <class R>
struct alignas(16) DevMesh {
  R lo[4];       // calcAABB (geom.nim:175-188), for the reference's mesh gate
  R hi[4];
  int32_t root;        // index into nodes, -1 for an empty mesh
  int32_t num_faces;
  int32_t normal_base; // offset (in faces) into normals
  int32_t pad;
};

// BVH2 node: both children's boxes in one 64-byte record (one scalar fetch
// tests two boxes). child n == 0: internal node index c (or c < 0: empty);
// n > 0: leaf with triangles [c, c + n) of the tris array.
struct alignas(16) BvhNode {
  float lo0[3], hi0[3];
  float lo1[3], hi1[3];
  int32_t c0, c1, n0, n1;
};
static_assert(sizeof(BvhNode) == 64, "BvhNode must be 64 bytes");

struct alignas(16) TriF32 {
  float v0[3];
  int32_t id;    // original face index (tie-break + normal lookup)
  float e1[3];
  float pad1;
  float e2[3];
  float pad2;
};
static_assert(sizeof(TriF32) == 48, "TriF32 must be 48 bytes");

// float32 kernel triangle (rt_fast.h tri_test): 64 bytes = ONE
// s_load_dwordx16. e2 = v2 - v0, e1n = -(v1 - v0), nn = -(e1 x e2), the
// cross product formed in float64 from the float64 edges, then rounded.
struct alignas(16) TriFast {
  float v0[3];
  int32_t id;    // original face index (tie-break + normal lookup)
  float e2[3];
  float pad0;
  float e1n[3];
  float pad1;
  float nn[3];
  float pad2;
};
static_assert(sizeof(TriFast) == 64, "TriFast must be 64 bytes");

struct alignas(16) TriF64 {
  double v0[3];
  double e1[3];
  double e2[3];
  int32_t id;
  int32_t pad;
};
static_assert(sizeof(TriF64) == 80, "TriF64 must be 80 bytes");

// A face's float64 shadow-ray record for one distant light (the parity
// kernel's light-cell searches, k_render_px64 mesh_lists): the values
// rayTriangleIntersectFast forms from the ray direction alone (geom.nim:
// 296-306: pvec = dir x v0v2, det = v0v1 . pvec, invDet = 1 / det) are fixed
// for a distant light's shadow rays, so k_build_sh64 forms them once per
// (light, grid entry) with tri_ref's operations on the light's object-space
// direction — the same bits a per-ray test forms — and a test reads them.
// Stored in light-grid entry order (a cell's faces are one contiguous run).
struct alignas(16) ShTri64 {
  double v0[3];
  double e1[3];
  double e2[3];
  double pvec[3];
  double det;
  double inv_det;
  int32_t id;
  int32_t pad[3];
};
static_assert(sizeof(ShTri64) == 128, "ShTri64 must be 128 bytes");

template <class R> struct TriOf;
template <> struct TriOf<float> { using type = TriF32; };
template <> struct TriOf<double> { using type = TriF64; };

// Kernel arguments (passed by value).
template <class R>
struct RenderParams {
  const DevObject<R>* objects;
  const DevLight<R>* lights;
  const DevMesh<R>* meshes;
  const BvhNode* nodes;
  const typename TriOf<R>::type* tris;
  const R* normals;
  float* fb;                       // output rows (see mode)
  unsigned long long* partials;    // [num_waves][kStatSlots]
  R c2w[16];
  R bg[4];
  R f;                             // tan(degToRad(fov) / 2)
  R aspect;                        // w / h
  R bias;
  R inv_len;                       // 1 / samples.len (renderer.nim:159)
  R sample_step;                   // grid: xs = ys = 1/m
  R sample_off;                    // grid: xoffs = yoffs = xs * 0.5
  int32_t nobj, nlight;
  int32_t width, height;
  int32_t aa_kind, grid_m, spp;
  int32_t max_depth;
  int32_t flags;
  int32_t max_iters;               // traversal bound: each node entered at most once
  int32_t shadow_mesh;             // the scene's only mesh object, or -1 (trace early exit)
  uint64_t seed;                   // stochastic samplers (rt_sampling.h)
  R* sample_scratch;               // per-lane sample tables [lanes][2][spp] (aa_kind >= 2)
  // work mapping: rows k in [0, nrows), columns j in [0, ncols), x = j*step.
  int32_t mode;                    // 0: y = y0 + k*step into full image; 1: bands
  int32_t y0, nrows, ncols, step, max_step;
  int32_t band_h, rank, world;
  int32_t lanes_per_px;            // L: lanes sharing one pixel's samples
  int32_t tile_x, tile_y;          // pixels per wave = tile_x * tile_y = 64 / L
  int32_t tiles_x;
  long long ngroups;               // tiles_x * tiles_y
  // this call's pixel records (rt_frame.h: list length + shadow skip bits
  // << 24), or nullptr: a pixel whose camera rays provably miss the mesh
  // skips its traversal for them, and for the shadow rays of the lights
  // whose skip bit is set (the camera level only)
  const uint32_t* pix_info;
  // k_render_px64 (one pixel per wave, float64): this call's camera-ray
  // face lists (rt_frame.h slots: min(n, 2^slot_lg) TriFast byte offsets
  // per pixel, n in pix_info; a TriFast offset o is TriF64 record
  // o / 64 - tri_rec0) and the scene's light grids (rt_bins.h), or nullptr:
  // the BVH serves those rays
  const int32_t* pix_slots;
  int32_t slot_lg;
  int32_t tri_rec0;
  const struct LightGrid* grids;
  const int32_t* grid_off;
  const int32_t* grid_ent;
  // k_render_px64's lean samples (rt_device.h px64_lean_sample): the plane of
  // a one-mesh + one-plane scene whose lights are all distant (<= 8) and whose
  // plane does not reflect, when this call has pixel records; -1 otherwise
  int32_t lean_plane;
  // the float64 shadow records (ShTri64) of the distant lights with a grid,
  // in grid entry order (index = G.ent_base + entry), or nullptr
  const ShTri64* sh64;
};

// ---- float32 performance-kernel records (rt_fast.h) -------------------------
// One 64-byte hot record per object: everything trace() needs, one s_load.
struct alignas(16) FObj {
  int32_t type, xf, mesh;
  int32_t root;   // mesh: BVH2 root node (FMesh.root), so a trace needs no FMesh fetch
  float t[3];     // world_to_object translation (XF_TRANSLATE)
  float r;        // sphere radius
  float lo[3];    // box vmin; mesh: its AABB (calcAABB, object space)
  float pad1;
  float hi[3];    // box vmax; mesh: its AABB
  float pad2;
};
static_assert(sizeof(FObj) == 64, "FObj must be 64 bytes");

// Shading data and the general transform, read only when needed.
struct alignas(16) FObjX {
  float w2o[12];     // world_to_object rows 0..2, column-major: w2o[c*3 + r]
  float o2w[9];      // object_to_world 3x3 (normals, not re-normalised)
  float albedo_pi[3];// albedo / PI (shader.nim:17)
  float refl;        // Material.reflection
  int32_t normal_base;
  int32_t pad[6];
};
static_assert(sizeof(FObjX) == 128, "FObjX must be 128 bytes");

struct alignas(16) FMesh {
  float lo[3];
  int32_t root;        // BVH2 root (index into nodes), -1 for an empty mesh
  float hi[3];
  int32_t normal_base;
};

// Light grid of one distant light for the float32 kernel (rt_bins.h): the
// mesh's faces binned by their projection along the object-space shadow
// direction. gu == 0: no grid for this light.
struct alignas(16) LightGrid {
  float e1[3];      // orthonormal basis of the plane orthogonal to the shadow direction
  float u0;
  float e2[3];
  float v0;
  float inv_h;      // cells per unit
  float rmax;       // |ro|_inf above this: the lane takes the BVH (float32 error bound)
  int32_t gu, gv;   // cells along e1 / e2
  int32_t off_base; // this grid's cell offsets start at FastParams.grid_off[off_base]
  int32_t ent_base; // added to its offsets: entries in FastParams.grid_ent
  int32_t pad[2];
};
static_assert(sizeof(LightGrid) == 64, "LightGrid must be 64 bytes");

struct alignas(16) FLight {
  int32_t type;
  float ci[3];   // color * intensity
  float v[3];    // dir (distant) / pos (point)
  float pad;
};

// FastParams.pix_info: the low 24 bits hold the pixel's list length (clamped;
// 0 = the camera rays cannot hit the mesh), bit 24 + l the shadow skip of
// light l (l < 8). kPixCount alone: nothing known about the pixel.
constexpr uint32_t kPixCount = 0x00FFFFFFu;

struct LTri;
struct FastParams {
  const FObj* objs;
  const FObjX* objx;
  const FMesh* meshes;
  const FLight* lights;
  const BvhNode* tree;              // nodes (child refs = byte offsets into tree) then TriFast records
  const float* normals;
  // pixel lists of the mesh (rt_frame.h): pixel y * width + x lists
  // min(n, 2^slot_lg) TriFast byte offsets at pix_slots[pix << slot_lg ..],
  // n = pix_cnt[pix] & kPixCount (n > 2^slot_lg: the list overflowed, the
  // pixel's camera rays take the BVH); pix_slots nullptr: BVH for camera rays
  const int32_t* pix_slots;
  const uint32_t* pix_cnt;
  const LightGrid* grids;          // per light, or nullptr: BVH for shadow rays
  const int32_t* grid_off;
  const int32_t* grid_ent;
  // object bins (rt_bins.h, scenes of 4..64 objects): 64-bit object masks
  const unsigned long long* obj_pix;   // per pixel (camera rays), or nullptr
  const LightGrid* obj_grids;          // per light (gu == 0: none), masks at obj_grid_mask[off_base + cell]
  const unsigned long long* obj_grid_mask;
  unsigned long long obj_off_grid;     // a safe lane outside an object grid: the unbounded objects
  const uint32_t* pix_info;        // per pixel: min(list length, kPixCount) | shadow skip bits << 24 (rt_bins.h),
                                   //   set when a wave holds one pixel; or nullptr
  float* fb;
  unsigned long long* partials;
  unsigned int* queue;             // kQueueShards heads (atomicAdd), zeroed at launch
  const int32_t* order;            // launch order of the pixel groups, or nullptr (identity)
  unsigned* cost;                  // per pixel group: its duration in cycles, or nullptr
  float cam[12];       // origin, C2W column 0, 1, 2 (xyz each)
  float cam_a, cam_b;  // cx = (px - cam_b) * cam_a, cam_b = w/2   (renderer.nim:39)
  float cam_c, cam_d;  // cy = (cam_d - py) * cam_c, cam_d = h/2   (renderer.nim:40)
  float bg[3];
  float bias;
  float inv_len;
  float sample_step, sample_off;
  int32_t nobj, nlight, width, height;
  int32_t aa_kind, grid_m, spp, max_depth, flags, shadow_mesh, shards, has_point_light, log2_tile_x;
  uint64_t seed;                   // stochastic samplers (rt_sampling.h)
  float inv_band_h;
  int32_t mode, y0, nrows, ncols, step, max_step, band_h, rank, world;
  int32_t lanes_per_px, log2_lanes, tile_x, tile_y, tiles_x, ngroups;
  int32_t log2_grid_m;             // akGrid m = 2^log2_grid_m (sample s = (s & (m-1), s >> log2)), or -1
  int32_t iters;                   // sample iterations per work item: ceil(spp / lanes_per_px)
  uint32_t tx_magic;               // g / tiles_x == (g * tx_magic) >> tx_shift for 0 <= g < 2^31
  int32_t tx_shift;
  int32_t stat_flush;              // work items between flushes of the 32-bit wave Stats counters
  int32_t slot_lg;                 // pixel list slots per pixel: 2^slot_lg
  // k_render_mix1's second list (lean pixels, k_render_lean1q items) and its shard count
  const int32_t* order2;
  int32_t ngroups2, shards2;
  // two-class launches: the entry counts of the lists at order / order2,
  // counted on the device by this call's k_frame_build2 (rt_frame.h), or
  // nullptr (the lists' lengths are ngroups / ngroups2, items of the kernel)
  const int32_t* list_n;
  const int32_t* list_n2;
  // reflection-ray compaction (k_render_wave): per-wave ray queues
  // (kReflQueue entries x kReflFields floats, field-major) and the
  // call's secondary radiance, 32.32 fixed point per pixel channel, indexed
  // (out_row * width + x) * 3 + c - sec_base * 3; nullptr: no compaction
  float* rq;
  long long* sec;
  int64_t sec_base;
  // shadow-ray records (LTri) of the distant lights whose bit is set in
  // lrec_mask: every float32 shadow test against the mesh for such a light —
  // cell lists, BVH leaves, batched or one-sample paths alike — reads the
  // face's record at lrec_base + light * lrec_stride + (its TriFast byte
  // offset), so every path forms the same t and the same verdict
  uint64_t lrec_base;
  int64_t lrec_stride;
  uint32_t lrec_mask;
  int32_t pad_lrec;
  // the same records in light-grid entry order: grid_rec[e] is the LTri of
  // the face grid_ent[e] names (for its grid's light), so a cell search reads
  // its faces' records straight from the cell's range — one load per step
  // instead of the entry, then the record it names; nullptr: via grid_ent
  const LTri* grid_rec;
};
// A face's shadow-ray test for one distant light (fixed direction d, mesh
// object space), prepared in float64 by the host (rtmi.cpp make_ltri): with
// c = (o - v0) x d the single-sided Moller-Trumbore test (geom.nim:283-336)
// is u = e2.c / det, v = -e1.c / det, t = (o - v0).nn / -det, nn = -(e1 x e2),
// det = nn.d — all three affine in the ray origin o alone:
//   u = p.o + cu, v = q.o + cv, t = tv.o + ct
// (p = (d x e2) / det, q = (d x -e1) / det, tv = nn / -det); a face with
// det < 1e-6 for this light can never pass (p = q = 0, cu = cv = -1). The
// hit test is then 9 FMAs and min(u, v, 1 - (u + v)) >= 0.
struct alignas(16) LTri {
  float p[3];
  float cu;
  float q[3];
  float cv;
  float tv[3];
  float ct;
  int32_t id;    // the face's index (TriFast.id)
  int32_t pad[3];
};
static_assert(sizeof(LTri) == 64, "LTri must be 64 bytes (one scalar load, TriFast-sized offsets)");
// reflection queue of a k_render_wave wave: up to 63 rays left over plus a
// pass's 64 new ones; fields ro xyz, rd xyz, weight, dst * 16 + depth
constexpr int kReflQueue = 128, kReflFields = 8;

enum : int32_t {
  STAT_PRIMARY = 0, STAT_TESTS = 1, STAT_HITS = 2, STAT_SHADOW = 3, STAT_REFL = 4,
  STAT_NODE_FETCH = 5, STAT_TRI_FETCH = 6, STAT_LANE_NODES = 7, STAT_LANE_TRIS = 8,
  STAT_GEN_FALLBACK = 9  // k_render_gen pixel groups re-rendered by the one-sample loop
};
// float32 kernel scene-feature subset index (rt_kernels_f32_part.hip): bit 0
// sphere, 1 box, 2 mesh, 3 general transform, 4 point light, 5 reflection,
// 6 stochastic sampling (a per-launch option, not a scene property)
enum : unsigned {
  SUB_SPHERE = 1u, SUB_BOX = 2u, SUB_MESH = 4u, SUB_XF_GENERAL = 8u, SUB_POINT = 16u, SUB_REFLECT = 32u,
  SUB_STOCHASTIC = 64u
};
// float32 kernel work queue: 64 head words, 128 B apart, zeroed per launch
constexpr int kQueueShards = 64, kQueueStride = 32;
// object-binned batches (k_render_fast, analytic scenes with distant lights,
// no reflection): samples per lane of one batch (rt_fast.h lean_batch<F, S,
// true>); the host's lane count gives a work item at least one batch
#ifndef RTMI_OBJ_BATCH
#define RTMI_OBJ_BATCH 4
#endif
constexpr int kObjBatch = RTMI_OBJ_BATCH;
// k_render_lean work item: a run of this many lean-list entries (the list
// padded with -1 to a whole number of runs), fetched with one scalar load
constexpr int kLeanRun = 4;

}  // namespace rtmi

// Launchers implemented by the precision-specific translation units.
extern "C" {
int rtmi_launch_render_f32(const rtmi::FastParams* p, unsigned subset, int blocks, size_t shmem, void* stream);
int rtmi_launch_wave_f32(const rtmi::FastParams* p, unsigned subset, int blocks, size_t shmem, void* stream);
int rtmi_wave_f32_blocks_per_cu(unsigned subset, size_t shmem);
int rtmi_launch_sec_add(float* fb, const long long* sec, size_t n, float scale, int num_cus, void* stream);
int rtmi_launch_render_f64(const rtmi::RenderParams<double>* p, int blocks, int px64, void* stream);
int rtmi_px64_blocks_per_cu(int px64);
int rtmi_px64_batch();
int rtmi_build_sh64(const rtmi::DevObject<double>* objects, int mesh_obj, const rtmi::DevLight<double>* lights,
                    int light, const int32_t* ent, int n, const rtmi::TriF64* tris, int tri_rec0,
                    rtmi::ShTri64* out, void* stream);
int rtmi_render_f32_blocks_per_cu(int count, unsigned subset, size_t shmem);
int rtmi_launch_lean_f32(const rtmi::FastParams* p, unsigned subset, int blocks, size_t shmem, void* stream);
int rtmi_lean_f32_blocks_per_cu(unsigned subset, size_t shmem);
int rtmi_launch_lean1_f32(const rtmi::FastParams* p, int nl, int lp, int blocks, void* stream);
int rtmi_lean1_f32_blocks_per_cu(int nl, int lp);
int rtmi_lean1_quads();
int rtmi_launch_gen1_f32(const rtmi::FastParams* p, int nl, int blocks, void* stream);
int rtmi_gen1_f32_blocks_per_cu(int nl);
int rtmi_launch_mix1_f32(const rtmi::FastParams* p, int nl, int lp, int blocks, void* stream);
int rtmi_mix1_f32_blocks_per_cu(int nl, int lp);
int rtmi_launch_gen_f32(const rtmi::FastParams* p, unsigned subset, int blocks, size_t shmem, void* stream);
int rtmi_gen_f32_blocks_per_cu(unsigned subset, size_t shmem);
int rtmi_launch_ppm_encode(const float* fb, long long n, int bits, int srgb, void* out, void* stream);
int rtmi_launch_rgba_encode(const float* fb, long long npix, unsigned int alpha, void* out, void* stream);
// Sets this thread's rt_last_error() text; returns code (rtmi.cpp).
int rtmi_fail_msg(int code, const char* msg);
int rtmi_launch_reduce_stats(const unsigned long long* partials, int num_waves,
                             unsigned long long* acc, void* stream);
int rtmi_launch_unshard(const float* gathered, float* fb, int width, int height, int band_h,
                        int world, void* stream);
}
