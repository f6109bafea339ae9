// rtmi.cpp — C-ABI (include/rtmi.h) of the MI355X trace/shade backend.
//
// Replaces the reference's renderLine / initRenderer
// (src/renderer/renderer.nim:162-215) behind plain C entry points: the scene
// is flattened and uploaded once (rt_scene_create), then whole frames, row
// ranges (the pool's scanline messages, src/raytracer.nim:25-32) or
// multi-GPU bands are rendered by the gfx950 kernels in rt_device.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <set>
#include <thread>
#include <string>
#include <vector>

#include "../../include/rtmi.h"
#include "rt_bins.h"
#include "rt_bvh.h"
#include "rt_common.h"
#include "rt_frame.h"

using namespace rtmi;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) return fail(RT_E_DEVICE, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  int alloc(size_t count) {
    release();
    if (count == 0) count = 1;
    hipError_t e = hipMalloc((void**)&p, count * sizeof(T));
    if (e != hipSuccess) {
      p = nullptr;
      return fail(RT_E_NOMEM, "hipMalloc(%zu bytes): %s", count * sizeof(T), hipGetErrorString(e));
    }
    n = count;
    return RT_OK;
  }
  int upload(const std::vector<T>& h) { return upload(h.data(), h.size()); }
  int upload(const T* h, size_t count) {
    int rc = alloc(count);
    if (rc != RT_OK) return rc;
    if (count) HIP_TRY(hipMemcpy(p, h, count * sizeof(T), hipMemcpyHostToDevice));
    return RT_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  size_t bytes() const { return n * sizeof(T); }
};

template <class R>
struct PrecisionData {
  DevBuf<DevObject<R>> objects;
  DevBuf<DevLight<R>> lights;
  DevBuf<DevMesh<R>> meshes;
  DevBuf<typename TriOf<R>::type> tris;
  DevBuf<R> normals;
  void release() {
    objects.release();
    lights.release();
    meshes.release();
    tris.release();
    normals.release();
  }
  size_t bytes() const {
    return objects.bytes() + lights.bytes() + meshes.bytes() + tris.bytes() + normals.bytes();
  }
};

struct FastData {
  DevBuf<FObj> objs;
  DevBuf<FObjX> objx;
  DevBuf<FMesh> meshes;
  DevBuf<FLight> lights;
  // the float32 kernel's BVH in ONE allocation: the nodes with child refs as
  // BYTE offsets into this buffer (inner child: its node, leaf: its first
  // TriFast record), then the TriFast records; one scalar base + a 32-bit
  // SGPR offset address every record (s_load ... soffset)
  DevBuf<BvhNode> tree;
  DevBuf<float> normals;
  void release() {
    objs.release();
    objx.release();
    meshes.release();
    lights.release();
    tree.release();
    normals.release();
  }
  size_t bytes() const {
    return objs.bytes() + objx.bytes() + meshes.bytes() + lights.bytes() + tree.bytes() + normals.bytes();
  }
};

bool is_pow2(int v) { return v > 0 && (v & (v - 1)) == 0; }

int device_of_current() {
  int d = -1;
  (void)hipGetDevice(&d);
  return d;
}

}  // namespace

// Pixel-list slots per pixel, 2^lg: RTMI_SLOT_LG (A/B knob) or -1 = by image size.
inline int slot_lg_env() {
  static const int v = [] {
    const char* e = rtmi::diag_env("RTMI_SLOT_LG");
    return e ? std::min(10, std::max(0, std::atoi(e))) : -1;
  }();
  return v;
}
// by image size: the most slots (a power of two, 2^kSlotLg .. 256) whose
// block stays within 2^27 entries
inline int slot_lg_for(int w, int h) {
  const unsigned long long npx = (unsigned long long)w * (unsigned long long)h;
  int lg = rtmi::kSlotLg;
  while (lg < 8 && (npx << (lg + 1)) <= (1ull << 27)) ++lg;
  // 4K and up: 128 (4.2 GB per buffer set at 4K). The 1M-face torus (C5)
  // lists up to 99 faces per pixel at 4K; with 64 slots its 64 fullest
  // pixels took the one-sample BVH loop at ~100x a mean pixel's cost, up
  // to ~12 ms of one wave — longer than a rank's whole call at N = 8, so
  // the 3 ranks holding the dearest of them ran 10-20 % long (rt_frame.h)
  if (npx >= (1ull << 22)) lg = std::max(lg, 7);
  return lg;
}

// LTri (rt_common.h) of face v for the shadow direction d (mesh object
// space, float64): p, q, tv rounded to float32 first, the constants formed
// from the ROUNDED vectors (u(v0) = 0 up to the float64 sum), so each affine
// function keeps its zero at the face's vertex.
static void make_ltri(const double v[3][3], const double d[3], int32_t face, LTri* out) {
  double e1[3], e2[3], cr[3], nn[3], p[3], q[3], me1[3];
  for (int k = 0; k < 3; ++k) {
    e1[k] = v[1][k] - v[0][k];
    e2[k] = v[2][k] - v[0][k];
    me1[k] = -e1[k];
  }
  rtmi::bg::cross3(e1, e2, cr);
  for (int k = 0; k < 3; ++k) nn[k] = -cr[k];
  const double det = rtmi::bg::dot3(nn, d);
  std::memset(out, 0, sizeof *out);
  out->id = face;
  if (!(det >= 1e-6)) {  // geom.nim:306: never passes for this light
    out->cu = out->cv = out->ct = -1.0f;
    return;
  }
  rtmi::bg::cross3(d, e2, p);
  rtmi::bg::cross3(d, me1, q);
  double pr[3], qr[3], tr[3];
  for (int k = 0; k < 3; ++k) {
    out->p[k] = (float)(p[k] / det);
    out->q[k] = (float)(q[k] / det);
    out->tv[k] = (float)(nn[k] / -det);
    pr[k] = out->p[k];
    qr[k] = out->q[k];
    tr[k] = out->tv[k];
  }
  out->cu = (float)-rtmi::bg::dot3(pr, v[0]);
  out->cv = (float)-rtmi::bg::dot3(qr, v[0]);
  out->ct = (float)-rtmi::bg::dot3(tr, v[0]);
}

struct rt_scene {
  std::mutex mu;
  int device = 0;
  int num_cus = 256;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;  // the last call's completion: its buffer set's `used` event (not owned)
  // two-class launches: the lean kernel runs on `aux`, forked from and
  // joined back into the caller's stream, so its waves take the general
  // kernel's slots as that kernel's waves drain (no tail between the two)
  hipStream_t aux = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  // Pipelined calls alternate between two sets of per-call buffers (Frame +
  // queue heads / Stats words): the call's camera-dependent build runs on
  // `bstream` (the device's highest stream priority), after only the call two
  // back that used the same set, so it overlaps the previous call's render
  // kernels; the render waits for its own build (Frame::built). The render's
  // persistent waves leave the build about one block per CU, so its first
  // launch stretches over the render and the other two follow it (rank 0 of
  // 8: 35 us of build in stream order, 23 us exposed when pipelined; a third
  // buffer set measured no better). A float32 call is pipelined when it renders at most
  // a third of the image (a multi-GPU rank's bands, a pool's scanlines: the
  // build is about fixed per call, the render shrinks with the launch); a
  // whole frame fills the GPU by itself and runs its build in stream order
  // (measured on C3: whole frame 0.906 ms serial vs 0.945 pipelined; rank 0
  // of 8 back to back 0.174 vs 0.163 ms). RTMI_PIPE=0 / 1 forces it off / on.
  hipStream_t bstream = nullptr;
  int pipe_mode = -1;    // RTMI_PIPE: -1 by launch size, 0 never, 1 always
  bool pipe = false;     // this call is pipelined
  // RT_FLAG_TIMING: call start, render kernels' start, call end
  hipEvent_t tev[3] = {nullptr, nullptr, nullptr};
  bool timed = false;
  int64_t last_lean = 0, last_general = 0;  // rt_scene_last_split
  int32_t last_lean_kind = 0;                // rt_scene_last_lean_kernel
  bool stats_kept = true;                    // the last call kept its Stats (no RT_FLAG_NO_STATS)
  // per-wave Stats rows of the last call not yet reduced into acc(): a call
  // whose caller does not read its Stats leaves them to the first reader
  // (rt_scene_last_stats / _last_counters), one launch fewer per call
  int32_t pending_reduce = 0;
  hipStream_t done_stream = nullptr;  // the stream `done` was last recorded on
  int64_t last_batched = 0, last_fallback = -1;  // rt_scene_last_batch
  int32_t nobj = 0, nlight = 0, nmesh = 0;
  int32_t shadow_mesh = -1;  // the only mesh object, or -1 (FastParams.shadow_mesh)
  int32_t lean64_plane = -1; // RenderParams.lean_plane of the scene (k_render_px64 lean samples)
  int32_t has_point_light = 0;
  unsigned f32_subset = 0;   // SUB_* feature bits of the scene (kernel specialisation)
  bool any_reflective = false;
  double fov = 50.0;
  double c2w[16];
  double bg[3];
  FastData f32;
  PrecisionData<double> f64;
  DevBuf<BvhNode> nodes;
  DevBuf<unsigned long long> partials;
  // float32 work-queue heads (two sets of kQueueShards * kQueueStride: the
  // general and the lean kernel), then the Stats accumulator: one buffer so
  // a call clears both with one fill
  DevBuf<unsigned int> queue, queue2;  // queue2: the other set's (swapped with fr2)
  static constexpr size_t kQueueWords = (size_t)2 * kQueueShards * kQueueStride;
  unsigned long long* acc() const { return reinterpret_cast<unsigned long long*>(queue.p + kQueueWords); }
  DevBuf<double> f64_tables;       // float64 kernel per-lane stochastic sample tables
  DevBuf<float> refl_queue;        // k_render_wave's per-wave ray queues
  DevBuf<long long> refl_sec;      // k_render_wave's per-pixel secondary radiance (32.32)
  struct Order {                   // one launch mapping's measured costs -> launch order
    std::array<int64_t, 17> key;
    DevBuf<unsigned> cost;         // cycles per pixel group, written by the measuring launch
    DevBuf<int32_t> perm;          // the expensive-first order, once built
    std::vector<int32_t> host_perm;  // the same order on the host (two-class launches split it)
    hipEvent_t measured = nullptr; // recorded after the measuring launch
    ~Order() {
      cost.release();
      perm.release();
      if (measured) (void)hipEventDestroy(measured);
    }
  };
  std::vector<std::unique_ptr<Order>> orders;  // most recently used first, at most 8
  // bins of the float32 kernel (rt_bins.h), for the scene's only mesh object
  std::vector<BinTri> bin_tris;    // its faces (object space) + TriFast byte offsets
  double mesh_o2w[16], mesh_w2o[16];
  bool binnable = false;
  DevBuf<LightGrid> grids;         // per light (gu == 0: none)
  // per light with a grid: every face's shadow-test record for that light's
  // fixed direction (rt_common.h LTri, leaf order, ntri per light)
  DevBuf<LTri> lrec;
  DevBuf<LTri> grec;               // lrec in light-grid entry order (FastParams.grid_rec)
  // the float64 shadow records in light-grid entry order (RenderParams.sh64),
  // built by the first float64 call that searches the grids
  DevBuf<ShTri64> sh64;
  bool sh64_ready = false;
  int64_t lrec_ntri = 0;
  uint32_t lrec_mask = 0;          // the lights that have records
  DevBuf<int32_t> grid_off, grid_ent;
  bool has_grids = false;
  // shadow skips (rt_bins.h): scenes of the one mesh and planes
  std::vector<GridOcc> grid_occ;   // per light (g.gu == 0: none)
  std::vector<LightGridHost> grid_host;  // per light: the cell lists + face boxes the shadow lists gather from
  std::vector<SkipPlane> skip_planes;
  bool skippable = false;
  // camera-dependent data of the float32 kernels (rt_frame.h): rebuilt on
  // the device by every render call; only the buffers outlive a call
  DevBuf<DevBinTri> bin_dev;       // the binned mesh's faces (float64, leaf order)
  double mesh_lo[3] = {0, 0, 0}, mesh_hi[3] = {0, 0, 0};  // its AABB (object space, calcAABB)
  DevBuf<int32_t> sat_dev;         // the light grids' occupancy prefix sums, back to back
  int64_t sat_off[8] = {};
  struct Frame {                   // per-call buffers of one image size
    int w = 0, h = 0;
    DevBuf<int32_t> cnt, slots, lean, heavy, ctr, orect;
    DevBuf<uint32_t> info;
    DevBuf<unsigned long long> omask, status;  // status: per-tile class counts (FrameLaunch.tile_cls)
    DevBuf<HugeFace> huge;
    DevBuf<unsigned char> tiles;   // per skip cell of a tile: shadow skips (k_frame_build1)
    int slot_lg = -1;              // slots allocated for 2^slot_lg entries per pixel (-1: none)
    int want_lg = slot_lg_env();   // test hook (rtmi_test_slot_lg) / RTMI_SLOT_LG; -1: by image size
    uint32_t calls = 0;            // build launches (their parity picks the huge-list counter)
    bool counted = false;          // the last launch's lean / general lists were counted on the device
    bool listed = false;           // the last launch built camera-ray lists
    hipEvent_t built = nullptr;    // recorded on bstream after this set's builds of a call
    hipEvent_t used = nullptr;     // recorded on the caller's stream at the end of a call that used this set
    bool used_rec = false;         // `used` has been recorded
    int id = 0;                    // which of the two sets (test hook)
    // forget the buffers: the next call re-allocates and re-zeroes them
    void invalidate() { w = h = 0; }
    size_t bytes() const {
      return cnt.bytes() + slots.bytes() + lean.bytes() + heavy.bytes() + ctr.bytes() + orect.bytes() +
             info.bytes() + omask.bytes() + status.bytes() + huge.bytes() + tiles.bytes();
    }
    void release() {
      cnt.release(); slots.release(); lean.release(); heavy.release(); ctr.release(); orect.release();
      info.release(); omask.release(); status.release(); huge.release(); tiles.release();
      slot_lg = -1;
      w = h = 0;
    }
  } fr, fr2;  // fr: this (or the last) call's set; fr2 the other one (swapped per call)
  // object bins (rt_bins.h ObjBox), scenes of 4..64 objects
  std::vector<ObjBox> obj_boxes;
  bool objbins = false;
  DevBuf<LightGrid> obj_grids;
  DevBuf<unsigned long long> obj_grid_mask;
  unsigned long long obj_off_grid = 0;
  bool has_obj_grids = false;
  DevBuf<DevObjBox> objbox_dev;
  DevBuf<float> fb_scratch;
  int max_waves = 0;
  int64_t num_triangles = 0, num_nodes = 0;
  int max_depth = 0;
  double build_ms = 0.0;

  ~rt_scene() {
    f32.release();
    f64.release();
    nodes.release();
    partials.release();
    queue.release();
    f64_tables.release();
    fb_scratch.release();
    grids.release();
    lrec.release();
    grec.release();
    grid_off.release();
    grid_ent.release();
    obj_grids.release();
    obj_grid_mask.release();
    fr.release();
    fr2.release();
    queue2.release();
    bin_dev.release();
    sat_dev.release();
    objbox_dev.release();
    if (fork) (void)hipEventDestroy(fork);
    for (hipEvent_t& e : tev)
      if (e) (void)hipEventDestroy(e);
    if (join) (void)hipEventDestroy(join);
    for (Frame* f : {&fr, &fr2}) {
      if (f->built) (void)hipEventDestroy(f->built);
      if (f->used) (void)hipEventDestroy(f->used);
    }
    if (bstream) (void)hipStreamDestroy(bstream);
    if (aux) (void)hipStreamDestroy(aux);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

int rtmi_fail_msg(int code, const char* msg) { return fail(code, "%s", msg ? msg : ""); }

extern "C" {

int rt_version(void) { return RTMI_ABI_VERSION; }

#ifndef RTMI_SOURCE_HASH
#define RTMI_SOURCE_HASH "unknown"
#endif
const char* rt_build_source_hash(void) { return RTMI_SOURCE_HASH; }

const char* rt_last_error(void) { return g_err.c_str(); }

int rt_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

int rt_init(int device) {
  const int n = rt_device_count();
  if (n <= 0) return fail(RT_E_DEVICE, "no HIP device visible");
  if (device < 0 || device >= n) return fail(RT_E_INVALID, "device %d out of range [0, %d)", device, n);
  HIP_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(RT_E_DEVICE, "device %d is %s; librtmi.so is built for gfx950 (MI355X) only", device,
                prop.gcnArchName);
  return RT_OK;
}

int rt_mat4_inverse(const double m_[16], double out[16]) {
  if (!m_ || !out) return fail(RT_E_INVALID, "null matrix");
  // GLM compute_inverse (cofactors times 1/determinant), m[c][r] = m_[c*4+r]
  auto m = [&](int c, int r) { return m_[c * 4 + r]; };
  const double Coef00 = m(2, 2) * m(3, 3) - m(3, 2) * m(2, 3);
  const double Coef02 = m(1, 2) * m(3, 3) - m(3, 2) * m(1, 3);
  const double Coef03 = m(1, 2) * m(2, 3) - m(2, 2) * m(1, 3);
  const double Coef04 = m(2, 1) * m(3, 3) - m(3, 1) * m(2, 3);
  const double Coef06 = m(1, 1) * m(3, 3) - m(3, 1) * m(1, 3);
  const double Coef07 = m(1, 1) * m(2, 3) - m(2, 1) * m(1, 3);
  const double Coef08 = m(2, 1) * m(3, 2) - m(3, 1) * m(2, 2);
  const double Coef10 = m(1, 1) * m(3, 2) - m(3, 1) * m(1, 2);
  const double Coef11 = m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2);
  const double Coef12 = m(2, 0) * m(3, 3) - m(3, 0) * m(2, 3);
  const double Coef14 = m(1, 0) * m(3, 3) - m(3, 0) * m(1, 3);
  const double Coef15 = m(1, 0) * m(2, 3) - m(2, 0) * m(1, 3);
  const double Coef16 = m(2, 0) * m(3, 2) - m(3, 0) * m(2, 2);
  const double Coef18 = m(1, 0) * m(3, 2) - m(3, 0) * m(1, 2);
  const double Coef19 = m(1, 0) * m(2, 2) - m(2, 0) * m(1, 2);
  const double Coef20 = m(2, 0) * m(3, 1) - m(3, 0) * m(2, 1);
  const double Coef22 = m(1, 0) * m(3, 1) - m(3, 0) * m(1, 1);
  const double Coef23 = m(1, 0) * m(2, 1) - m(2, 0) * m(1, 1);
  const double Fac0[4] = {Coef00, Coef00, Coef02, Coef03};
  const double Fac1[4] = {Coef04, Coef04, Coef06, Coef07};
  const double Fac2[4] = {Coef08, Coef08, Coef10, Coef11};
  const double Fac3[4] = {Coef12, Coef12, Coef14, Coef15};
  const double Fac4[4] = {Coef16, Coef16, Coef18, Coef19};
  const double Fac5[4] = {Coef20, Coef20, Coef22, Coef23};
  const double Vec0[4] = {m(1, 0), m(0, 0), m(0, 0), m(0, 0)};
  const double Vec1[4] = {m(1, 1), m(0, 1), m(0, 1), m(0, 1)};
  const double Vec2[4] = {m(1, 2), m(0, 2), m(0, 2), m(0, 2)};
  const double Vec3[4] = {m(1, 3), m(0, 3), m(0, 3), m(0, 3)};
  double inv[4][4];
  const double SignA[4] = {+1, -1, +1, -1}, SignB[4] = {-1, +1, -1, +1};
  for (int i = 0; i < 4; ++i) {
    inv[0][i] = (Vec1[i] * Fac0[i] - Vec2[i] * Fac1[i] + Vec3[i] * Fac2[i]) * SignA[i];
    inv[1][i] = (Vec0[i] * Fac0[i] - Vec2[i] * Fac3[i] + Vec3[i] * Fac4[i]) * SignB[i];
    inv[2][i] = (Vec0[i] * Fac1[i] - Vec1[i] * Fac3[i] + Vec3[i] * Fac5[i]) * SignA[i];
    inv[3][i] = (Vec0[i] * Fac2[i] - Vec1[i] * Fac4[i] + Vec2[i] * Fac5[i]) * SignB[i];
  }
  const double Row0[4] = {inv[0][0], inv[1][0], inv[2][0], inv[3][0]};
  double Dot0[4];
  for (int i = 0; i < 4; ++i) Dot0[i] = m(0, i) * Row0[i];
  const double Dot1 = (Dot0[0] + Dot0[1]) + (Dot0[2] + Dot0[3]);
  if (Dot1 == 0.0 || !std::isfinite(Dot1)) return fail(RT_E_INVALID, "singular matrix");
  const double one_over_det = 1.0 / Dot1;
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 4; ++r) out[c * 4 + r] = inv[c][r] * one_over_det;
  return RT_OK;
}

int rt_load_geom(const char* path, int64_t* num_triangles, double* vertices) {
  if (!path || !num_triangles) return fail(RT_E_INVALID, "null argument");
  FILE* f = std::fopen(path, "rb");
  if (!f) return fail(RT_E_IO, "cannot open %s", path);
  int32_t n = 0;
  if (std::fread(&n, 4, 1, f) != 1 || n < 0) {
    std::fclose(f);
    return fail(RT_E_IO, "%s: bad .geom header", path);
  }
  if (!vertices) {
    std::fclose(f);
    *num_triangles = n;
    return RT_OK;
  }
  if (*num_triangles < n) {
    std::fclose(f);
    return fail(RT_E_INVALID, "buffer holds %lld triangles, file has %d", (long long)*num_triangles, n);
  }
  std::vector<float> buf((size_t)n * 9);
  const size_t got = buf.empty() ? 0 : std::fread(buf.data(), sizeof(float), buf.size(), f);
  std::fclose(f);
  if (got != buf.size()) return fail(RT_E_IO, "%s: truncated (%zu of %zu floats)", path, got, buf.size());
  for (size_t i = 0; i < buf.size(); ++i) vertices[i] = (double)buf[i];
  *num_triangles = n;
  return RT_OK;
}

int rt_band_rows(int32_t height, int32_t band_h, int32_t world, int32_t* out_rows) {
  if (!out_rows || height <= 0 || band_h <= 0 || world <= 0) return fail(RT_E_INVALID, "bad band geometry");
  const int32_t nbands = (height + band_h - 1) / band_h;
  *out_rows = ((nbands + world - 1) / world) * band_h;
  return RT_OK;
}

}  // extern "C"

namespace {

bool affine(const double* m) { return m[3] == 0.0 && m[7] == 0.0 && m[11] == 0.0 && m[15] == 1.0; }

// fn(begin, end) over [0, n) in contiguous chunks on up to 16 host threads
// (scene setup of million-face meshes: per-face record packing).
template <class Fn>
void parallel_for(int64_t n, Fn fn) {
  const int64_t kGrain = 1 << 15;
  const int hw = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const int nt = (int)std::min<int64_t>(hw, (n + kGrain - 1) / kGrain);
  if (nt <= 1) {
    if (n > 0) fn((int64_t)0, n);
    return;
  }
  std::vector<std::thread> pool;
  pool.reserve((size_t)nt);
  for (int t = 0; t < nt; ++t) pool.emplace_back([=, &fn] { fn(n * t / nt, n * (t + 1) / nt); });
  for (std::thread& th : pool) th.join();
}

// Identity / pure translation / general (float32 fast paths, DevObject.xf).
// Translation requires BOTH matrices to have an identity 3x3 block, so the
// normal transform (object_to_world * n) is the identity too.
int32_t classify_xf(const double* w2o, const double* o2w) {
  bool lin_id = true;
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) {
      const double id = c == r ? 1.0 : 0.0;
      if (w2o[c * 4 + r] != id || o2w[c * 4 + r] != id) lin_id = false;
    }
  if (!lin_id) return XF_GENERAL;
  if (w2o[12] == 0.0 && w2o[13] == 0.0 && w2o[14] == 0.0) return XF_IDENTITY;
  return XF_TRANSLATE;
}

template <class R>
void fill_precision(const rt_scene_desc* d, const std::vector<std::vector<double>>& normals,
                    const std::vector<BvhResult>& bvhs, const std::vector<int32_t>& node_base,
                    const std::vector<std::vector<double>>& aabbs, std::vector<DevObject<R>>& objs,
                    std::vector<DevLight<R>>& lights, std::vector<DevMesh<R>>& meshes,
                    std::vector<typename TriOf<R>::type>* tris, std::vector<R>& nrm) {
  objs.assign((size_t)d->num_objects, DevObject<R>{});
  for (int i = 0; i < d->num_objects; ++i) {
    const rt_object_desc& s = d->objects[i];
    DevObject<R>& o = objs[(size_t)i];
    for (int k = 0; k < 16; ++k) {
      o.w2o[k] = (R)s.world_to_object[k];
      o.o2w[k] = (R)s.object_to_world[k];
    }
    o.prm[0] = (R)(s.type == RT_SPHERE ? s.radius : s.box_min[0]);
    o.prm[1] = (R)s.box_min[1];
    o.prm[2] = (R)s.box_min[2];
    o.prm[4] = (R)s.box_max[0];
    o.prm[5] = (R)s.box_max[1];
    o.prm[6] = (R)s.box_max[2];
    for (int k = 0; k < 3; ++k) o.albedo[k] = (R)s.albedo[k];
    o.albedo[3] = (R)s.reflection;
    // albedo / PI in R, one correctly rounded IEEE division as the kernel's
    // (and the oracle's, rt_oracle.c shade) per-sample quotient
    for (int k = 0; k < 3; ++k) o.albp[k] = (R)s.albedo[k] / (R)3.14159265358979323846;
    o.type = s.type;
    o.mesh = s.type == RT_MESH ? s.mesh : 0;
    o.xf = classify_xf(s.world_to_object, s.object_to_world);
  }
  lights.assign((size_t)d->num_lights, DevLight<R>{});
  for (int i = 0; i < d->num_lights; ++i) {
    const rt_light_desc& s = d->lights[i];
    DevLight<R>& l = lights[(size_t)i];
    // color * intensity, computed in float64 like light.nim:50,57
    for (int k = 0; k < 3; ++k) l.ci[k] = (R)(s.color[k] * s.intensity);
    for (int k = 0; k < 3; ++k) l.v[k] = (R)(s.type == RT_POINT_LIGHT ? s.pos[k] : s.dir[k]);
    l.type = s.type == RT_POINT_LIGHT ? LIGHT_POINT : LIGHT_DISTANT;
  }
  meshes.assign((size_t)d->num_meshes, DevMesh<R>{});
  int64_t total = 0;
  for (int m = 0; m < d->num_meshes; ++m) total += d->meshes[m].num_faces;
  if (tris) tris->assign((size_t)total, typename TriOf<R>::type{});
  nrm.resize((size_t)total * 3);
  int32_t normal_base = 0;
  for (int m = 0; m < d->num_meshes; ++m) {
    const rt_mesh_desc& md = d->meshes[m];
    DevMesh<R>& dm = meshes[(size_t)m];
    for (int k = 0; k < 3; ++k) {
      dm.lo[k] = (R)aabbs[(size_t)m][k];
      dm.hi[k] = (R)aabbs[(size_t)m][3 + k];
    }
    dm.num_faces = (int32_t)md.num_faces;
    dm.normal_base = normal_base;
    dm.root = bvhs[(size_t)m].nodes.empty() ? -1 : node_base[(size_t)m];
    const std::vector<int32_t>& order = bvhs[(size_t)m].order;
    if (tris) {
      typename TriOf<R>::type* out = tris->data() + normal_base;
      parallel_for((int64_t)order.size(), [&](int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i) {
          const int32_t face = order[(size_t)i];
          typename TriOf<R>::type& t = out[i];
          const int32_t* fi = &md.faces[3 * (size_t)face];
          const double* v0 = &md.vertices[3 * (size_t)fi[0]];
          const double* v1 = &md.vertices[3 * (size_t)fi[1]];
          const double* v2 = &md.vertices[3 * (size_t)fi[2]];
          for (int k = 0; k < 3; ++k) {
            t.v0[k] = (R)v0[k];
            t.e1[k] = (R)(v1[k] - v0[k]);  // v0v1 exactly as geom.nim:286-288
            t.e2[k] = (R)(v2[k] - v0[k]);  // v0v2 exactly as geom.nim:292-294
          }
          t.id = face;
        }
      });
    }
    const std::vector<double>& src = normals[(size_t)m];
    R* dst = nrm.data() + 3 * (size_t)normal_base;
    parallel_for((int64_t)src.size(), [&](int64_t b, int64_t e) {
      for (int64_t i = b; i < e; ++i) dst[i] = (R)src[(size_t)i];
    });
    normal_base += (int32_t)md.num_faces;
  }
  // pad so a kernel may read kLeafMax records from any leaf start
  if (tris)
    for (int k = 0; k < kLeafMax - 1; ++k) {
      typename TriOf<R>::type t{};
      t.id = -1;
      tris->push_back(t);
    }
}

// float32 kernel records (rt_common.h FObj/FObjX/FMesh/FLight).
void fill_fast_records(const rt_scene_desc* d, const std::vector<DevMesh<float>>& dm, std::vector<FObj>& fo,
                       std::vector<FObjX>& fx, std::vector<FMesh>& fm, std::vector<FLight>& fl) {
  const double kPi = 3.14159265358979323846;
  fo.assign((size_t)d->num_objects, FObj{});
  fx.assign((size_t)d->num_objects, FObjX{});
  for (int i = 0; i < d->num_objects; ++i) {
    const rt_object_desc& s = d->objects[i];
    FObj& o = fo[(size_t)i];
    FObjX& x = fx[(size_t)i];
    o.type = s.type;
    o.xf = classify_xf(s.world_to_object, s.object_to_world);
    o.mesh = s.type == RT_MESH ? s.mesh : 0;
    for (int k = 0; k < 3; ++k) {
      o.t[k] = (float)s.world_to_object[12 + k];
      o.lo[k] = (float)(s.type == RT_MESH ? dm[(size_t)s.mesh].lo[k] : s.box_min[k]);
      o.hi[k] = (float)(s.type == RT_MESH ? dm[(size_t)s.mesh].hi[k] : s.box_max[k]);
    }
    // byte offset of the root node in FastData.tree
    o.root = s.type == RT_MESH && dm[(size_t)s.mesh].root >= 0 ? dm[(size_t)s.mesh].root * (int32_t)sizeof(BvhNode) : -1;
    o.r = (float)s.radius;
    for (int c = 0; c < 4; ++c)
      for (int r = 0; r < 3; ++r) x.w2o[c * 3 + r] = (float)s.world_to_object[c * 4 + r];
    for (int c = 0; c < 3; ++c)
      for (int r = 0; r < 3; ++r) x.o2w[c * 3 + r] = (float)s.object_to_world[c * 4 + r];
    for (int k = 0; k < 3; ++k) x.albedo_pi[k] = (float)(s.albedo[k] / kPi);
    x.refl = (float)s.reflection;
    x.normal_base = s.type == RT_MESH ? dm[(size_t)s.mesh].normal_base : 0;
  }
  fm.assign(dm.size(), FMesh{});
  for (size_t m = 0; m < dm.size(); ++m) {
    for (int k = 0; k < 3; ++k) {
      fm[m].lo[k] = dm[m].lo[k];
      fm[m].hi[k] = dm[m].hi[k];
    }
    fm[m].root = dm[m].root;
    fm[m].normal_base = dm[m].normal_base;
  }
  fl.assign((size_t)d->num_lights, FLight{});
  for (int i = 0; i < d->num_lights; ++i) {
    const rt_light_desc& s = d->lights[i];
    fl[(size_t)i].type = s.type == RT_POINT_LIGHT ? LIGHT_POINT : LIGHT_DISTANT;
    for (int k = 0; k < 3; ++k) {
      fl[(size_t)i].ci[k] = (float)(s.color[k] * s.intensity);
      fl[(size_t)i].v[k] = (float)(s.type == RT_POINT_LIGHT ? s.pos[k] : s.dir[k]);
    }
  }
}

}  // namespace

extern "C" int rt_scene_create(const rt_scene_desc* d, rt_scene** out_scene) {
  if (!d || !out_scene) return fail(RT_E_INVALID, "null argument");
  *out_scene = nullptr;
  if (d->num_objects < 0 || d->num_lights < 0 || d->num_meshes < 0)
    return fail(RT_E_INVALID, "negative counts");
  if ((d->num_objects > 0 && !d->objects) || (d->num_lights > 0 && !d->lights) ||
      (d->num_meshes > 0 && !d->meshes))
    return fail(RT_E_INVALID, "null array with nonzero count");
  if (!affine(d->camera_to_world)) return fail(RT_E_UNSUPPORTED, "camera_to_world is not affine");
  const auto t0 = std::chrono::steady_clock::now();
  // RTMI_SETUP_PROFILE=1: per-phase wall times of scene setup on stderr
  static const bool profile = rtmi::diag_env("RTMI_SETUP_PROFILE") != nullptr;
  auto tp = t0;
  const auto mark = [&](const char* phase) {
    if (!profile) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[rtmi setup] %-22s %9.3f ms\n", phase,
                 std::chrono::duration<double, std::milli>(now - tp).count());
    tp = now;
  };
  bool any_reflective = false;
  for (int i = 0; i < d->num_objects; ++i) {
    const rt_object_desc& o = d->objects[i];
    if (o.type < RT_SPHERE || o.type > RT_MESH) return fail(RT_E_INVALID, "object %d: bad type %d", i, o.type);
    if (o.type == RT_MESH && (o.mesh < 0 || o.mesh >= d->num_meshes))
      return fail(RT_E_INVALID, "object %d: mesh index %d out of range", i, o.mesh);
    if (!affine(o.object_to_world) || !affine(o.world_to_object))
      return fail(RT_E_UNSUPPORTED, "object %d: non-affine transform", i);
    if (o.reflection > 0.0) any_reflective = true;
  }
  for (int i = 0; i < d->num_lights; ++i)
    if (d->lights[i].type != RT_DISTANT_LIGHT && d->lights[i].type != RT_POINT_LIGHT)
      return fail(RT_E_INVALID, "light %d: bad type", i);
  if (d->bvh_builder != RT_BVH_SAH && d->bvh_builder != RT_BVH_PLOC)
    return fail(RT_E_INVALID, "bad bvh_builder %d", d->bvh_builder);
  int dev = device_of_current();
  if (dev < 0 || rt_device_count() <= 0) return fail(RT_E_DEVICE, "no HIP device (call rt_init)");
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, dev));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(RT_E_DEVICE, "device %d is %s; librtmi.so is built for gfx950 only", dev, prop.gcnArchName);
  std::vector<std::vector<double>> normals((size_t)d->num_meshes), aabbs((size_t)d->num_meshes);
  std::vector<BvhResult> bvhs((size_t)d->num_meshes);
  // device copies of every mesh's arrays: the device builder and the
  // triangle-record packing (rt_bvh_gpu.hip) read them
  std::vector<DevBuf<double>> d_verts((size_t)d->num_meshes);
  std::vector<DevBuf<int32_t>> d_faces((size_t)d->num_meshes);
  struct FreeAll {
    std::vector<DevBuf<double>>& v;
    std::vector<DevBuf<int32_t>>& f;
    ~FreeAll() {
      for (auto& b : v) b.release();
      for (auto& b : f) b.release();
    }
  } free_all{d_verts, d_faces};
  std::vector<int32_t> node_base((size_t)d->num_meshes, 0);
  int64_t ntri = 0, nnodes = 0;
  int maxdepth = 0;
  std::vector<BvhNode> all_nodes;
  for (int m = 0; m < d->num_meshes; ++m) {
    const rt_mesh_desc& md = d->meshes[m];
    if (md.num_faces < 0 || md.num_vertices < 0 || (md.num_faces > 0 && (!md.faces || !md.vertices)))
      return fail(RT_E_INVALID, "mesh %d: bad arrays", m);
    for (int64_t k = 0; k < md.num_faces * 3; ++k)
      if (md.faces[k] < 0 || md.faces[k] >= md.num_vertices)
        return fail(RT_E_INVALID, "mesh %d: face index %d out of range", m, md.faces[k]);
    // face normals: given, or calcNormals (src/loaders/obj.nim:65-84)
    std::vector<double>& nr = normals[(size_t)m];
    nr.resize((size_t)md.num_faces * 3);
    parallel_for(md.num_faces, [&](int64_t fb, int64_t fe) {
    for (int64_t fidx = fb; fidx < fe; ++fidx) {
      if (md.normals) {
        for (int k = 0; k < 3; ++k) nr[3 * (size_t)fidx + k] = md.normals[3 * fidx + k];
        continue;
      }
      const double* p0 = &md.vertices[3 * (size_t)md.faces[3 * fidx + 0]];
      const double* p1 = &md.vertices[3 * (size_t)md.faces[3 * fidx + 1]];
      const double* p2 = &md.vertices[3 * (size_t)md.faces[3 * fidx + 2]];
      const double ax = p1[0] - p0[0], ay = p1[1] - p0[1], az = p1[2] - p0[2];
      const double bx = p2[0] - p0[0], by = p2[1] - p0[1], bz = p2[2] - p0[2];
      const double cx = ay * bz - az * by, cy = az * bx - ax * bz, cz = ax * by - ay * bx;
      double dd = 0.0;
      dd = dd + cx * cx;
      dd = dd + cy * cy;
      dd = dd + cz * cz;
      const double len = std::sqrt(dd);
      nr[3 * (size_t)fidx + 0] = cx / len;
      nr[3 * (size_t)fidx + 1] = cy / len;
      nr[3 * (size_t)fidx + 2] = cz / len;
    }
    });
    // calcAABB (geom.nim:175-188) over every vertex
    std::vector<double>& bb = aabbs[(size_t)m];
    bb = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (int64_t v = 0; v < md.num_vertices; ++v)
      for (int k = 0; k < 3; ++k) {
        const double x = md.vertices[3 * v + k];
        if (x < bb[(size_t)k]) bb[(size_t)k] = x;
        if (x > bb[3 + (size_t)k]) bb[3 + (size_t)k] = x;
      }
    mark("normals + bounds");
    int urc;
    if ((urc = d_verts[(size_t)m].upload(md.vertices, (size_t)md.num_vertices * 3)) ||
        (urc = d_faces[(size_t)m].upload(md.faces, (size_t)md.num_faces * 3)))
      return urc;
    mark("mesh upload");
    const char* err = "BVH build failed";
    BvhBuildParams prm;
    const bool ok = d->bvh_builder == RT_BVH_PLOC
                        ? build_bvh_device(d_verts[(size_t)m].p, d_faces[(size_t)m].p, md.num_faces, prm,
                                           &bvhs[(size_t)m], &err)
                        : build_bvh(md.vertices, md.faces, md.num_faces, prm, &bvhs[(size_t)m], &err);
    if (!ok) return fail(d->bvh_builder == RT_BVH_PLOC ? RT_E_DEVICE : RT_E_INVALID, "mesh %d: %s", m, err);
    mark("bvh build");
    node_base[(size_t)m] = (int32_t)all_nodes.size();
    for (BvhNode nd : bvhs[(size_t)m].nodes) {
      if (nd.n0 == 0 && nd.c0 >= 0) nd.c0 += node_base[(size_t)m];
      if (nd.n1 == 0 && nd.c1 >= 0) nd.c1 += node_base[(size_t)m];
      if (nd.n0 > 0) nd.c0 += (int32_t)ntri;
      if (nd.n1 > 0) nd.c1 += (int32_t)ntri;
      all_nodes.push_back(nd);
    }
    ntri += md.num_faces;
    nnodes += (int64_t)bvhs[(size_t)m].nodes.size();
    maxdepth = std::max(maxdepth, bvhs[(size_t)m].max_depth);
  }
  if (ntri > INT32_MAX / 2) return fail(RT_E_UNSUPPORTED, "too many triangles");
  // the float32 kernel addresses its tree with signed 32-bit byte offsets
  if ((nnodes + ntri + kLeafMax) * (int64_t)sizeof(BvhNode) > (int64_t)INT32_MAX)
    return fail(RT_E_UNSUPPORTED, "%lld BVH nodes + %lld triangles exceed the float32 tree's 2 GiB offset range",
                (long long)nnodes, (long long)ntri);


  std::unique_ptr<rt_scene> s(new rt_scene());
  s->device = dev;
  s->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  s->nobj = d->num_objects;
  {
    int n_mesh_obj = 0;
    for (int i = 0; i < d->num_objects; ++i)
      if (d->objects[i].type == RT_MESH) {
        ++n_mesh_obj;
        s->shadow_mesh = i;
      }
    if (n_mesh_obj != 1) s->shadow_mesh = -1;
  }
  s->nlight = d->num_lights;
  for (int i = 0; i < d->num_lights; ++i)
    if (d->lights[i].type == RT_POINT_LIGHT) s->has_point_light = 1;
  s->nmesh = d->num_meshes;
  s->any_reflective = any_reflective;
  // scene features -> the float32 kernel specialisation (rt_kernels_f32_part.hip)
  s->f32_subset = 0;
  for (int i = 0; i < d->num_objects; ++i) {
    const rt_object_desc& ob = d->objects[i];
    if (ob.type == RT_SPHERE) s->f32_subset |= SUB_SPHERE;
    if (ob.type == RT_BOX) s->f32_subset |= SUB_BOX;
    if (ob.type == RT_MESH) s->f32_subset |= SUB_MESH;
    if (classify_xf(ob.world_to_object, ob.object_to_world) == XF_GENERAL) s->f32_subset |= SUB_XF_GENERAL;
  }
  if (s->has_point_light) s->f32_subset |= SUB_POINT;
  if (any_reflective) s->f32_subset |= SUB_REFLECT;
  s->fov = d->fov;
  std::memcpy(s->c2w, d->camera_to_world, sizeof s->c2w);
  std::memcpy(s->bg, d->bg_color, sizeof s->bg);
  HIP_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
  HIP_TRY(hipStreamCreateWithFlags(&s->aux, hipStreamNonBlocking));
  HIP_TRY(hipEventCreateWithFlags(&s->fork, hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&s->join, hipEventDisableTiming));
  for (hipEvent_t& e : s->tev) HIP_TRY(hipEventCreate(&e));
  {
    // the build stream at the highest priority (rank 0 of 8 back to back:
    // 0.163 -> 0.161 ms); RTMI_PIPE_PRIO=0: the default priority (A/B)
    int lo = 0, hi = 0;
    const char* pe = rtmi::diag_env("RTMI_PIPE_PRIO");
    if (!(pe && std::atoi(pe) == 0) && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess)
      HIP_TRY(hipStreamCreateWithPriority(&s->bstream, hipStreamNonBlocking, hi));
    else
      HIP_TRY(hipStreamCreateWithFlags(&s->bstream, hipStreamNonBlocking));
  }
  {
    // `built` only orders the build stream before the caller's stream on this
    // device: a device-scope release (no system-scope cache writeback) is
    // enough. `used` doubles as `done`, which the host waits on before
    // reading device memory and peers copy behind: system scope.
    // RTMI_EVENT_SCOPE (A/B): 0 both system scope, 2 both device scope.
    const char* es = rtmi::diag_env("RTMI_EVENT_SCOPE");
    const int scope = es && *es ? std::atoi(es) : 1;
    const unsigned fb = hipEventDisableTiming | (scope >= 1 ? hipEventReleaseToDevice : 0u);
    const unsigned fu = hipEventDisableTiming | (scope >= 2 ? hipEventReleaseToDevice : 0u);
    for (rt_scene::Frame* f : {&s->fr, &s->fr2}) {
      HIP_TRY(hipEventCreateWithFlags(&f->built, fb));
      HIP_TRY(hipEventCreateWithFlags(&f->used, fu));
    }
  }
  s->done = s->fr.used;
  s->fr2.id = 1;
  {
    const char* e = std::getenv("RTMI_PIPE");
    s->pipe_mode = e && *e ? (std::atoi(e) != 0 ? 1 : 0) : -1;
  }
  {
    std::vector<DevObject<float>> o;
    std::vector<DevLight<float>> l;
    std::vector<DevMesh<float>> m;
    std::vector<float> n;
    fill_precision<float>(d, normals, bvhs, node_base, aabbs, o, l, m, nullptr, n);
    mark("fp32 records");
    std::vector<FObj> fo;
    std::vector<FObjX> fx;
    std::vector<FMesh> fm;
    std::vector<FLight> fl;
    fill_fast_records(d, m, fo, fx, fm, fl);
    int rc;
    if ((rc = s->f32.objs.upload(fo)) || (rc = s->f32.objx.upload(fx)) || (rc = s->f32.meshes.upload(fm)) ||
        (rc = s->f32.lights.upload(fl)) || (rc = s->f32.normals.upload(n)))
      return rc;
    mark("fp32 upload");
  }
  {
    std::vector<DevObject<double>> o;
    std::vector<DevLight<double>> l;
    std::vector<DevMesh<double>> m;
    std::vector<double> n;
    fill_precision<double>(d, normals, bvhs, node_base, aabbs, o, l, m, nullptr, n);
    mark("fp64 records");
    int rc;
    if ((rc = s->f64.objects.upload(o)) || (rc = s->f64.lights.upload(l)) || (rc = s->f64.meshes.upload(m)) ||
        (rc = s->f64.normals.upload(n)))
      return rc;
  }
  mark("fp64 upload");
  {
    // triangle records in BVH leaf order, packed on the device; the float64
    // array carries kLeafMax - 1 padding records (id -1) so a kernel may
    // read kLeafMax records from any leaf start
    int rc;
    if ((rc = s->f32.tree.alloc((size_t)(nnodes + ntri))) || (rc = s->f64.tris.alloc((size_t)ntri + kLeafMax - 1)))
      return rc;
    TriFast* f32_tris = reinterpret_cast<TriFast*>(s->f32.tree.p + nnodes);
    std::vector<TriF64> pad((size_t)kLeafMax - 1);
    for (TriF64& t : pad) {
      std::memset(&t, 0, sizeof t);
      t.id = -1;
    }
    HIP_TRY(hipMemcpy(s->f64.tris.p + ntri, pad.data(), pad.size() * sizeof(TriF64), hipMemcpyHostToDevice));
    int64_t base = 0;
    for (int m = 0; m < d->num_meshes; ++m) {
      const int64_t nf = d->meshes[m].num_faces;
      DevBuf<int32_t> order;
      if ((rc = order.upload(bvhs[(size_t)m].order))) return rc;
      const bool ok = pack_triangles_device(d_verts[(size_t)m].p, d_faces[(size_t)m].p, order.p, nf,
                                            f32_tris + base, s->f64.tris.p + base, s->stream);
      HIP_TRY(hipStreamSynchronize(s->stream));
      order.release();
      if (!ok) return fail(RT_E_DEVICE, "mesh %d: triangle packing failed", m);
      base += nf;
    }
  }
  mark("triangle packing");
  int rc = s->nodes.upload(all_nodes);
  if (rc) return rc;
  {  // float32 tree: child refs -> byte offsets (leaves: past the nnodes node records)
    std::vector<BvhNode> fn(all_nodes);
    const int32_t kB = (int32_t)sizeof(BvhNode);
    for (BvhNode& nd : fn) {
      nd.c0 = (nd.n0 > 0 ? (int32_t)nnodes + nd.c0 : nd.c0) * kB;
      nd.c1 = (nd.n1 > 0 ? (int32_t)nnodes + nd.c1 : nd.c1) * kB;
    }
    if (!fn.empty())
      HIP_TRY(hipMemcpy(s->f32.tree.p, fn.data(), fn.size() * sizeof(BvhNode), hipMemcpyHostToDevice));
  }
  if (s->shadow_mesh >= 0) {  // bins of the only mesh object (rt_bins.h)
    const rt_object_desc& ob = d->objects[s->shadow_mesh];
    const int m = ob.mesh;
    const rt_mesh_desc& md = d->meshes[m];
    int64_t base = 0;
    for (int k = 0; k < m; ++k) base += d->meshes[k].num_faces;
    const std::vector<int32_t>& order = bvhs[(size_t)m].order;
    s->bin_tris.resize(order.size());
    parallel_for((int64_t)order.size(), [&](int64_t b, int64_t e) {
      for (int64_t i = b; i < e; ++i) {
        BinTri& t = s->bin_tris[(size_t)i];
        const int32_t* fi = &md.faces[3 * (size_t)order[(size_t)i]];
        for (int v = 0; v < 3; ++v)
          for (int k = 0; k < 3; ++k) t.v[v][k] = md.vertices[3 * (size_t)fi[v] + k];
        t.rec = (int32_t)((nnodes + base + i) * (int64_t)sizeof(TriFast));
        t.face = order[(size_t)i];
      }
    });
    std::memcpy(s->mesh_o2w, ob.object_to_world, sizeof s->mesh_o2w);
    std::memcpy(s->mesh_w2o, ob.world_to_object, sizeof s->mesh_w2o);
    s->binnable = !s->bin_tris.empty();
    static_assert(sizeof(BinTri) == sizeof(DevBinTri) && offsetof(BinTri, rec) == offsetof(DevBinTri, rec),
                  "BinTri and DevBinTri share one layout");
    if (s->binnable) {
      if ((rc = s->bin_dev.alloc(s->bin_tris.size()))) return rc;
      HIP_TRY(hipMemcpy(s->bin_dev.p, s->bin_tris.data(), s->bin_tris.size() * sizeof(BinTri), hipMemcpyHostToDevice));
      for (int k = 0; k < 3; ++k) {
        s->mesh_lo[k] = aabbs[(size_t)m][k];
        s->mesh_hi[k] = aabbs[(size_t)m][3 + k];
      }
    }
    // light grids of the distant lights
    std::vector<LightGrid> gh((size_t)std::max(1, d->num_lights), LightGrid{});
    s->grid_occ.assign((size_t)d->num_lights, GridOcc{});
    s->grid_host.assign((size_t)d->num_lights, LightGridHost{});
    std::vector<int32_t> goff, gent;
    bool any = false;
    for (int li = 0; s->binnable && li < d->num_lights; ++li) {
      if (d->lights[li].type == RT_POINT_LIGHT) continue;
      LightGridHost lg;
      const char* why = "";
      if (!build_light_grid(s->bin_tris, s->mesh_w2o, d->lights[li].dir, &lg, &why)) continue;
      if ((int64_t)goff.size() + (int64_t)lg.off.size() > INT32_MAX ||
          (int64_t)gent.size() + (int64_t)lg.ent.size() > INT32_MAX)
        break;
      lg.g.off_base = (int32_t)goff.size();
      lg.g.ent_base = (int32_t)gent.size();
      goff.insert(goff.end(), lg.off.begin(), lg.off.end());
      gent.insert(gent.end(), lg.ent.begin(), lg.ent.end());
      gh[(size_t)li] = lg.g;
      grid_occupancy(lg, &s->grid_occ[(size_t)li]);
      s->grid_host[(size_t)li] = std::move(lg);
      s->grid_occ[(size_t)li].lists = &s->grid_host[(size_t)li];
      any = true;
    }
    if (any) {
      if ((rc = s->grids.upload(gh)) || (rc = s->grid_off.upload(goff)) || (rc = s->grid_ent.upload(gent))) return rc;
      s->has_grids = true;
      // the shadow-test records of the lights with a grid (the float32
      // kernels' every shadow ray to such a light tests these, on every path)
      {
        const size_t nt = (size_t)ntri;  // indexed like the TriFast records: byte offset / 64 - nnodes
        // every slot starts as the culled sentinel make_ltri writes for a face
        // that can never pass (u = v = t = -1): an all-zero record would read
        // as a hit at t = 0 (u = v = 0 passes min(u, v, 1-u-v) >= 0) if a
        // future path read a slot of another mesh's face or of a light with
        // no grid
        LTri culled;
        std::memset(&culled, 0, sizeof culled);
        culled.cu = culled.cv = culled.ct = -1.0f;
        culled.id = -1;
        std::vector<LTri> lr((size_t)d->num_lights * nt, culled);
        for (int li = 0; li < d->num_lights; ++li) {
          if (gh[(size_t)li].gu <= 0) continue;
          const double* dir = d->lights[li].dir;
          double sd[3], ld[3];
          for (int k = 0; k < 3; ++k) sd[k] = -dir[k];
          bg::xform_dir(s->mesh_w2o, sd, ld);  // the shadow direction in the mesh's object space
          parallel_for((int64_t)nt, [&](int64_t b, int64_t e) {
            for (int64_t i = b; i < e; ++i) {
              const BinTri& t = s->bin_tris[(size_t)i];
              const int64_t slot = (int64_t)t.rec / (int64_t)sizeof(TriFast) - nnodes;
              make_ltri(t.v, ld, t.face, &lr[(size_t)li * nt + (size_t)slot]);
            }
          });
        }
        if ((rc = s->lrec.upload(lr))) return rc;
        s->lrec_ntri = (int64_t)nt;
        // the cell-ordered copy: entry e of light li's grid -> its face's record
        std::vector<LTri> gr(gent.size(), culled);
        for (int li = 0; li < d->num_lights; ++li) {
          if (gh[(size_t)li].gu <= 0) continue;
          const LightGridHost& lg = s->grid_host[(size_t)li];
          const size_t e0 = (size_t)gh[(size_t)li].ent_base, ne = lg.ent.size();
          parallel_for((int64_t)ne, [&](int64_t b, int64_t e) {
            for (int64_t k = b; k < e; ++k) {
              const int64_t slot = (int64_t)gent[e0 + (size_t)k] / (int64_t)sizeof(TriFast) - nnodes;
              gr[e0 + (size_t)k] = lr[(size_t)li * nt + (size_t)slot];
            }
          });
        }
        if ((rc = s->grec.upload(gr))) return rc;
        for (int li = 0; li < d->num_lights && li < 32; ++li)
          if (gh[(size_t)li].gu > 0) s->lrec_mask |= 1u << li;
      }
      // shadow skips: every other object a plane
      s->skippable = true;
      for (int i = 0; i < d->num_objects; ++i) {
        const rt_object_desc& o = d->objects[i];
        if (i == s->shadow_mesh) continue;
        SkipPlane sp;
        s->skippable = s->skippable && o.type == RT_PLANE;
        std::memcpy(sp.o2w, o.object_to_world, sizeof sp.o2w);
        std::memcpy(sp.w2o, o.world_to_object, sizeof sp.w2o);
        s->skip_planes.push_back(sp);
      }
      if (!s->skippable) s->skip_planes.clear();
      // k_render_px64's lean samples: one mesh + one non-reflective plane,
      // distant lights only (each with a skip bit)
      s->lean64_plane = -1;
      if (s->skippable && s->shadow_mesh >= 0 && d->num_objects == 2 && d->num_lights >= 1 && d->num_lights <= 8) {
        const int pl = 1 - s->shadow_mesh;
        bool ok = d->objects[pl].type == RT_PLANE && !(d->objects[pl].reflection > 0.0);
        for (int li = 0; li < d->num_lights; ++li) ok = ok && d->lights[li].type != RT_POINT_LIGHT;
        if (ok) s->lean64_plane = pl;
      }
      // the occupancy prefix sums the per-call shadow skips read (rt_frame.h)
      std::vector<int32_t> sat;
      for (int li = 0; li < std::min(8, d->num_lights); ++li) {
        s->sat_off[li] = (int64_t)sat.size();
        sat.insert(sat.end(), s->grid_occ[(size_t)li].sat.begin(), s->grid_occ[(size_t)li].sat.end());
      }
      if (sat.empty()) sat.push_back(0);
      if ((rc = s->sat_dev.upload(sat))) return rc;
    }
    mark("light grids");
  }
  if (d->num_objects >= 4 && d->num_objects <= 64) {  // object bins (rt_bins.h)
    s->obj_boxes.assign((size_t)d->num_objects, ObjBox{});
    for (int i = 0; i < d->num_objects; ++i) {
      const rt_object_desc& ob = d->objects[i];
      ObjBox& b = s->obj_boxes[(size_t)i];
      double lo[3], hi[3], o2w[16];
      b.always = ob.type == RT_PLANE || rt_mat4_inverse(ob.world_to_object, o2w) != RT_OK;
      if (b.always) continue;
      for (int k = 0; k < 3; ++k) {
        lo[k] = ob.type == RT_SPHERE ? -std::fabs(ob.radius) : ob.type == RT_BOX ? ob.box_min[k] : aabbs[(size_t)ob.mesh][k];
        hi[k] = ob.type == RT_SPHERE ? std::fabs(ob.radius) : ob.type == RT_BOX ? ob.box_max[k] : aabbs[(size_t)ob.mesh][3 + k];
        b.lo[k] = INFINITY;
        b.hi[k] = -INFINITY;
      }
      // the world box of the object box, through the inverse of the
      // world_to_object the kernel transforms rays with
      for (int c = 0; c < 8; ++c) {
        const double q[3] = {(c & 1) ? hi[0] : lo[0], (c & 2) ? hi[1] : lo[1], (c & 4) ? hi[2] : lo[2]};
        for (int r = 0; r < 3; ++r) {
          const double w = o2w[0 * 4 + r] * q[0] + o2w[1 * 4 + r] * q[1] + o2w[2 * 4 + r] * q[2] + o2w[3 * 4 + r];
          b.corner[c][r] = w;
          b.lo[r] = std::min(b.lo[r], w);
          b.hi[r] = std::max(b.hi[r], w);
        }
      }
      for (int k = 0; k < 3; ++k)
        if (!std::isfinite(b.lo[k]) || !std::isfinite(b.hi[k])) b.always = true;
    }
    s->objbins = true;
    std::vector<DevObjBox> ob((size_t)d->num_objects);
    for (int i = 0; i < d->num_objects; ++i) {
      const ObjBox& b = s->obj_boxes[(size_t)i];
      for (int k = 0; k < 3; ++k) {
        ob[(size_t)i].lo[k] = b.lo[k];
        ob[(size_t)i].hi[k] = b.hi[k];
      }
      ob[(size_t)i].always = b.always ? 1 : 0;
      ob[(size_t)i].pad = 0;
    }
    if ((rc = s->objbox_dev.upload(ob))) return rc;
    std::vector<LightGrid> gh((size_t)std::max(1, d->num_lights), LightGrid{});
    std::vector<unsigned long long> gm;
    bool any = false;
    for (int li = 0; li < d->num_lights; ++li) {
      if (d->lights[li].type == RT_POINT_LIGHT) continue;
      ObjGridHost og;
      const char* why = "";
      if (!build_object_light_grid(s->obj_boxes, d->lights[li].dir, &og, &why)) continue;
      if ((int64_t)gm.size() + (int64_t)og.masks.size() > INT32_MAX) break;
      og.g.off_base = (int32_t)gm.size();
      gm.insert(gm.end(), og.masks.begin(), og.masks.end());
      gh[(size_t)li] = og.g;
      s->obj_off_grid = og.off_grid;  // the same set (the unbounded objects) for every light
      any = true;
    }
    if (any) {
      if ((rc = s->obj_grids.upload(gh)) || (rc = s->obj_grid_mask.upload(gm))) return rc;
      s->has_obj_grids = true;
    }
    mark("object bins");
  }
  s->max_waves = s->num_cus * 8 * 4;  // 8 blocks of 4 waves per CU at most
  // two kernels per two-class launch: their waves' partial counters side by side
  if ((rc = s->partials.alloc((size_t)2 * s->max_waves * kStatSlots))) return rc;
  if ((rc = s->queue.alloc(rt_scene::kQueueWords + 2 * (size_t)kStatSlots))) return rc;  // heads + Stats
  HIP_TRY(hipMemset(s->queue.p, 0, s->queue.bytes()));
  if ((rc = s->queue2.alloc(s->queue.n))) return rc;
  HIP_TRY(hipMemset(s->queue2.p, 0, s->queue2.bytes()));
  HIP_TRY(hipDeviceSynchronize());
  mark("nodes + buffers");
  s->num_triangles = ntri;
  s->num_nodes = nnodes;
  s->max_depth = maxdepth;
  s->build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *out_scene = s.release();
  return RT_OK;
}

extern "C" int rt_scene_destroy(rt_scene* s) {
  if (!s) return fail(RT_E_INVALID, "null scene");
  int prev = device_of_current();
  if (prev != s->device) (void)hipSetDevice(s->device);
  {
    // a call still inside the library on this scene (another thread) holds
    // s->mu: wait for it to leave before the scene goes. The caller must not
    // start new calls on a scene it destroys (rtmi.h); the Python / Nim
    // caches keep a per-scene count of calls in flight for that
    std::lock_guard<std::mutex> lk(s->mu);
    if (s->done) (void)hipEventSynchronize(s->done);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    if (s->bstream) (void)hipStreamSynchronize(s->bstream);
  }
  delete s;
  if (prev >= 0 && prev != -1) (void)hipSetDevice(prev);
  return RT_OK;
}

extern "C" int rt_scene_get_info(const rt_scene* s, rt_scene_info* out) {
  if (!s || !out) return fail(RT_E_INVALID, "null argument");
  out->num_objects = s->nobj;
  out->num_lights = s->nlight;
  out->num_meshes = s->nmesh;
  out->num_triangles = s->num_triangles;
  out->num_bvh_nodes = s->num_nodes;
  out->max_bvh_depth = s->max_depth;
  out->device = s->device;
  // everything the scene holds on the device: the geometry and BVH of both
  // precisions, the light grids and bins, and the per-call buffer sets
  // (fr / fr2 are the bulk at 4K)
  std::lock_guard<std::mutex> lk(const_cast<rt_scene*>(s)->mu);
  out->device_bytes = (int64_t)(s->f32.bytes() + s->f64.bytes() + s->nodes.bytes() + s->partials.bytes() + s->sh64.bytes() +
                                s->queue.bytes() + s->queue2.bytes() + s->f64_tables.bytes() +
                                s->fb_scratch.bytes() + s->grids.bytes() + s->grid_off.bytes() +
                                s->grid_ent.bytes() + s->obj_grids.bytes() + s->obj_grid_mask.bytes() +
                                s->bin_dev.bytes() + s->sat_dev.bytes() + s->objbox_dev.bytes() +
                                s->lrec.bytes() + s->grec.bytes() + s->fr.bytes() + s->fr2.bytes());
  out->build_ms = s->build_ms;
  return RT_OK;
}

extern "C" int rt_scene_set_camera(rt_scene* s, const double c2w[16], double fov_deg) {
  if (!s || !c2w) return fail(RT_E_INVALID, "null argument");
  for (int k = 0; k < 16; ++k)
    if (!std::isfinite(c2w[k])) return fail(RT_E_INVALID, "camera_to_world[%d] is not finite", k);
  if (!(fov_deg > 0.0 && fov_deg < 180.0)) return fail(RT_E_INVALID, "fov %g outside (0, 180)", fov_deg);
  std::lock_guard<std::mutex> lk(s->mu);
  const int prev = device_of_current();
  if (prev != s->device) (void)hipSetDevice(s->device);
  // earlier calls may still read the launch orders measured for the old camera
  const hipError_t e = hipEventSynchronize(s->done);
  std::memcpy(s->c2w, c2w, sizeof s->c2w);
  s->fov = fov_deg;
  s->orders.clear();    // measured per-group costs (launch order) too
  if (prev >= 0 && prev != s->device) (void)hipSetDevice(prev);
  if (e != hipSuccess) return fail(RT_E_DEVICE, "waiting for the scene's earlier calls: %s", hipGetErrorString(e));
  return RT_OK;
}

namespace {

struct Mapping {
  int mode, y0, nrows, ncols, step, max_step, band_h, rank, world;
};

int check_options(const rt_scene* s, const rt_options* o) {
  if (!o) return fail(RT_E_INVALID, "null options");
  if (o->width <= 0 || o->height <= 0 || o->width > 65536 || o->height > 65536)
    return fail(RT_E_INVALID, "bad image size %dx%d", o->width, o->height);
  if (o->aa_kind < RT_AA_NONE || o->aa_kind > RT_AA_CORRELATED_MULTI_JITTERED)
    return fail(RT_E_INVALID, "bad aa_kind %d", o->aa_kind);
  if (o->aa_kind != RT_AA_NONE && (o->grid_size < 1 || o->grid_size > 256))
    return fail(RT_E_INVALID, "grid_size %d out of range [1, 256]", o->grid_size);
  if (o->precision != RT_FP32 && o->precision != RT_FP64) return fail(RT_E_INVALID, "bad precision");
  // the float32 kernel builds a (multi-)jittered table in LDS per pixel:
  // 8 KB per wave at m = 32
  if (o->precision == RT_FP32 && o->aa_kind >= RT_AA_MULTI_JITTERED && o->grid_size > 32)
    return fail(RT_E_UNSUPPORTED, "float32 (multi-)jittered sampling supports grid_size <= 32 (got %d)",
                o->grid_size);
  if (s->any_reflective && o->max_ray_depth > kMaxShadeLevels - 1)
    return fail(RT_E_UNSUPPORTED, "max_ray_depth %d > %d with reflective materials", o->max_ray_depth,
                kMaxShadeLevels - 1);
  return RT_OK;
}

// The float32 kernel specialisation of a launch: the scene's features plus
// stochastic sampling when the options ask for it.
unsigned f32_subset(const rt_scene* s, const rt_options* o) {
  return s->f32_subset | (o->aa_kind >= RT_AA_JITTERED ? SUB_STOCHASTIC : 0u);
}

// Lanes per pixel of a float32 launch (a power of two, <= 64): as many as
// the samples fill; scenes of spheres / boxes / planes with distant lights
// and no reflection (k_render_fast's object-binned batches) use fewer, so a
// work item holds at least one batch of kObjBatch = 4 iterations (C2: 64 spp
// -> 16 lanes, 4 pixels per wave), but not fewer than 16 (8 for a batch of
// 8). The count does not depend on the binning / batching flags, so
// RT_FLAG_NO_BINNING and RT_FLAG_NO_OBJ_BATCH frames stay bit-identical (the
// same samples per lane, summed in the same order).
int f32_lanes(const rt_scene* s, const rt_options* o, int spp) {
  // diagnostic A/B: RTMI_MAX_LANES caps the lanes per pixel
  static const int max_lanes = rtmi::diag_env("RTMI_MAX_LANES") ? std::atoi(rtmi::diag_env("RTMI_MAX_LANES")) : 64;
  int L = 1;
  while (L * 2 <= std::min(std::min(spp, 64), std::max(1, max_lanes))) L *= 2;
  const unsigned sub = f32_subset(s, o);
  const bool ob_batch = !(sub & (SUB_MESH | SUB_REFLECT | SUB_POINT)) && (sub & (SUB_SPHERE | SUB_BOX));
  const int lmin = kObjBatch > 4 ? 8 : 16;  // <= 8 pixels per wave (the kernel's object-mask union)
  while (ob_batch && L > lmin && spp / L < kObjBatch) L /= 2;
  return L;
}

// Dynamic LDS of a float32 launch: the (multi-)jittered tables, 64/L
// pixels per wave x 2 x spp floats x 4 waves per block.
size_t f32_table_lds(const rt_scene* s, const rt_options* o) {
  if (o->precision != RT_FP32 || o->aa_kind < RT_AA_MULTI_JITTERED) return 0;
  const int spp = o->grid_size * o->grid_size;
  const int L = f32_lanes(s, o, spp);
  return (size_t)4 * (64 / L) * 2 * (size_t)spp * sizeof(float);
}

// Lanes per pixel (L), pixels per wave tile, number of wave groups, grid.
struct Plan {
  int L, log2L, tx, ty, tiles_x, ngroups, blocks;
};

Plan plan_mapping(const rt_scene* s, const rt_options* o, const Mapping& mp, int spp) {
  Plan pl{};
  // float64 parity mode keeps the reference's sequential sample sum (one
  // lane per pixel); float32 spreads a pixel's samples over up to 64 lanes.
  int L = 1, lg = 0;
  if (o->precision == RT_FP32) {
    L = f32_lanes(s, o, spp);
    while ((1 << lg) < L) ++lg;
  }
  const int P = 64 / L;
  int tx = 1, ty = 1;
  switch (P) {
    case 64: tx = 8; ty = 8; break;
    case 32: tx = 8; ty = 4; break;
    case 16: tx = 4; ty = 4; break;
    case 8: tx = 4; ty = 2; break;
    case 4: tx = 2; ty = 2; break;
    case 2: tx = 2; ty = 1; break;
    default: tx = 1; ty = 1; break;
  }
  pl.L = L;
  pl.log2L = lg;
  pl.tx = tx;
  pl.ty = ty;
  pl.tiles_x = (mp.ncols + tx - 1) / tx;
  const long long tiles_y = (mp.nrows + ty - 1) / ty;
  const long long ng = (long long)pl.tiles_x * tiles_y;
  pl.ngroups = (int)std::min<long long>(ng, INT32_MAX);
  const long long want = (ng + 3) / 4;
  long long cap = s->max_waves / 4;
  if (o->precision == RT_FP32) {  // work-queue kernel: launch what is resident
    const int per_cu = rtmi_render_f32_blocks_per_cu((o->flags & RT_FLAG_COUNT_TRAVERSAL) ? 1 : 0,
                                                     f32_subset(s, o), f32_table_lds(s, o));
    cap = std::min<long long>(cap, (long long)per_cu * s->num_cus);
  }
  pl.blocks = (int)std::max(1LL, std::min<long long>(want, cap));
  return pl;
}

// Launch order of the pixel groups: expensive first, from measured costs.
// Per-pixel cost varies ~20x (sky vs bunny + its shadows) and the work queue
// hands groups out in index order, so a launch ends when the wave that drew
// the last expensive group finishes it: a fixed ~0.2 ms on every C3 launch
// (a group at 256 spp is one pixel, up to ~0.2 ms of a wave's time), 2.5 %
// of a frame on one GPU and ~17 % of each rank's share on 8. The first
// launch of a mapping (image size, rows, bands, sampling) runs in screen
// order and records each group's duration (s_memtime); later launches of the
// same mapping hand groups out longest-first (LPT), so the tail is cheap
// groups — for launches short enough that the tail matters (below). Scheduling only: every launch traces every ray, and the image and
// Stats do not depend on the order. Off with RT_FLAG_NO_REORDER.
constexpr long long kLptGroupsPerWave = 96;

struct OrderUse {
  const int32_t* order = nullptr;  // FastParams.order
  unsigned* cost = nullptr;        // FastParams.cost (the measuring launch)
  rt_scene::Order* entry = nullptr;
  const std::vector<int32_t>* host_order = nullptr;  // the order on the host
};

int order_policy() {
  static const int v = [] {
    // tuning knob: 0 off, 1 LPT, 2 LPT in half octaves, 3 heavy then light
    // (split at the RTMI_ORDER_P cost quantile, screen order within each),
    // 4 = 3 with the light part longest-first. Off by default (round 3): the
    // costs are measured on an earlier frame of the same camera, and no
    // camera-dependent data is carried from one call to the next; the
    // two-class launches already hand out the expensive (general) pixels
    // before the cheap (lean) ones.
    const char* e = rtmi::diag_env("RTMI_ORDER");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

double order_quantile() {
  static const double v = [] {
    const char* e = rtmi::diag_env("RTMI_ORDER_P");
    return e ? std::atof(e) : 0.5;
  }();
  return v;
}

OrderUse group_order(rt_scene* s, const rt_options* o, const Mapping& mp, const FastParams& p, int blocks) {
  OrderUse u;
  const int policy = order_policy();
  // LPT only where the tail outweighs locality: with >= ~128 groups per
  // resident wave, screen order's spatial coherence (neighbouring pixels
  // share BVH paths in the scalar caches) is worth more than the tail (C3:
  // whole frame 8.15 ms screen vs 8.36 LPT; half frame equal; quarter 2.22
  // vs 2.10; eighth 1.23 vs 1.07; 1/64 0.34 vs 0.26)
  const long long waves = (long long)blocks * 4;
  if (policy == 0 || (o->flags & RT_FLAG_NO_REORDER) || p.ngroups < waves || p.ngroups > kLptGroupsPerWave * waves)
    return u;
  const std::array<int64_t, 17> key = {o->width,   o->height,  mp.mode,     mp.y0,       mp.nrows,  mp.ncols,
                                       mp.step,    mp.max_step, mp.band_h,  mp.rank,     mp.world,  p.tile_x,
                                       p.tile_y,   p.ngroups,   o->aa_kind, o->grid_size, o->max_ray_depth};
  size_t i = 0;
  while (i < s->orders.size() && s->orders[i]->key != key) ++i;
  if (i == s->orders.size()) {  // new mapping: measure it
    std::unique_ptr<rt_scene::Order> e(new rt_scene::Order());
    e->key = key;
    if (e->cost.alloc((size_t)p.ngroups) != RT_OK ||
        hipEventCreateWithFlags(&e->measured, hipEventDisableTiming) != hipSuccess)
      return u;
    s->orders.insert(s->orders.begin(), std::move(e));
    if (s->orders.size() > 8) s->orders.pop_back();
    u.cost = s->orders[0]->cost.p;
    u.entry = s->orders[0].get();
    return u;
  }
  std::rotate(s->orders.begin(), s->orders.begin() + (long)i, s->orders.begin() + (long)i + 1);
  rt_scene::Order& e = *s->orders[0];
  if (!e.perm.p) {
    std::vector<unsigned> c((size_t)p.ngroups);
    if (hipEventSynchronize(e.measured) != hipSuccess ||
        hipMemcpy(c.data(), e.cost.p, c.size() * sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess)
      return u;
    // stable counting sort, most expensive bucket first
    constexpr int kBuckets = 4096;
    unsigned cmax = 1;
    for (unsigned v : c) cmax = std::max(cmax, v);
    unsigned split = 0;  // policies 3/4: costs above this are "heavy"
    if (policy >= 3) {
      std::vector<unsigned> t(c);
      const size_t q = std::min(t.size() - 1, (size_t)(order_quantile() * (double)t.size()));
      std::nth_element(t.begin(), t.begin() + (long)q, t.end());
      split = t[q];
    }
    std::vector<uint16_t> bucket(c.size());
    std::vector<int32_t> start(kBuckets + 1, 0);
    for (size_t g = 0; g < c.size(); ++g) {
      int b;
      if (policy == 3) {
        b = c[g] > split ? kBuckets - 1 : 0;
      } else if (policy == 4) {
        b = c[g] > split ? kBuckets - 1 : (int)((uint64_t)c[g] * (kBuckets - 2) / std::max(split, 1u));
      } else if (policy == 2) {  // half-octave classes: keeps screen order within a class
        const unsigned v = std::max(c[g], 1u);
        const int l = 31 - __builtin_clz(v);
        b = 2 * l + (l > 0 ? (int)((v >> (l - 1)) & 1u) : 0);
      } else {
        b = (int)((uint64_t)c[g] * (kBuckets - 1) / cmax);
      }
      b = kBuckets - 1 - b;
      bucket[g] = (uint16_t)b;
      ++start[(size_t)b + 1];
    }
    for (int b = 0; b < kBuckets; ++b) start[(size_t)b + 1] += start[(size_t)b];
    std::vector<int32_t> perm(c.size());
    for (size_t g = 0; g < c.size(); ++g) perm[(size_t)start[bucket[g]]++] = (int32_t)g;
    if (e.perm.upload(perm) != RT_OK) return u;
    e.host_perm.swap(perm);
    e.cost.release();
  }
  u.order = e.perm.p;
  u.host_order = &e.host_perm;
  return u;
}

// ---- camera-dependent data, rebuilt by every float32 render call (rt_frame.h)

FrameRows frame_rows(const Mapping& mp, int height) {
  FrameRows r;
  r.mode = mp.mode;
  r.y0 = mp.y0;
  r.nrows = mp.nrows;
  r.step = mp.step;
  r.band_h = mp.band_h;
  r.rank = mp.rank;
  r.world = mp.world;
  r.height = height;
  return r;
}

// The per-call buffers of one image size (contents are rebuilt by each call).
int frame_buffers(rt_scene* s, int w, int h, hipStream_t st) {
  rt_scene::Frame& f = s->fr;
  const bool lists = s->binnable && !s->bin_tris.empty();
  // slots per pixel: 2^want_lg when set (test hook / RTMI_SLOT_LG), else
  // as many as 2^27 entries (512 MB) allow, 32 to 256: a mesh's per-pixel
  // lists are longer the fewer pixels it covers (the bunny: 28 faces at most
  // at 1080p, past 32 for 7 % of its pixels at 320x180); a pixel past its
  // slots takes the BVH (exact, slower)
  int lg = f.want_lg >= 0 ? f.want_lg : slot_lg_for(w, h);
  // slot indices are 32-bit (pixel << lg + slot, int in the kernels): a
  // requested lg (test hook / diagnostic) is clamped to keep the block below
  // 2^31 entries
  while (lg > 0 && (((unsigned long long)w * (unsigned long long)h) << lg) + kBinPad >= (1ull << 31)) --lg;
  if (f.w == w && f.h == h && (!lists || f.slot_lg == lg)) return RT_OK;
  // an earlier call may still read the old buffers: `st` (the build stream)
  // waits on the last call that used this set (its render kernels, and the
  // aux-stream kernels joined into it), so this one wait covers them all
  HIP_TRY(hipStreamSynchronize(st));
  const size_t npx = (size_t)w * (size_t)h;
  int rc;
  f.invalidate();
  if ((rc = f.cnt.alloc(npx + 1)) || (rc = f.info.alloc(npx)) || (rc = f.lean.alloc(npx + 64)) ||
      (rc = f.heavy.alloc(npx)) || (rc = f.ctr.alloc(FC_WORDS)) ||
      (rc = f.tiles.alloc((size_t)rtmi_frame_skip_cells(w, h))) ||
      (rc = f.status.alloc((size_t)rtmi_frame_tile_bytes(w, h))))
    return rc;
  if (s->objbins && ((rc = f.omask.alloc(npx)) || (rc = f.orect.alloc(kObjRectInts)))) return rc;
  if (lists) {
    // the slots hold valid record offsets from the start (the list search
    // reads up to kBinPad entries past a list's end)
    const size_t ns = (npx << lg) + kBinPad;
    if ((rc = f.slots.alloc(ns)) || (rc = f.huge.alloc(kHugeCap))) return rc;
    HIP_TRY(hipMemsetD32Async(f.slots.p, s->bin_tris[0].rec, ns, st));
    f.slot_lg = lg;
  }
  // the per-pixel counters are zero between calls (k_frame_build2 zeroes
  // the ones a call used)
  // (stream-ordered before the call's build launches on the same stream)
  HIP_TRY(hipMemsetAsync(f.cnt.p, 0, f.cnt.bytes(), st));
  HIP_TRY(hipMemsetAsync(f.ctr.p, 0, f.ctr.bytes(), st));
  HIP_TRY(hipMemsetAsync(f.info.p, 0, f.info.bytes(), st));  // (only read for the call's pixels; defined for the test hook)
  f.w = w;
  f.h = h;
  return RT_OK;
}

// The call's pixel-record / list parameters (RecordsLaunch) for the
// launch's pixels.
void records_launch(rt_scene* s, const rt_options* o, const Mapping& mp, const FastParams& p, bool records,
                    bool split, RecordsLaunch& r) {
  std::memset(&r, 0, sizeof r);
  r.mode = mp.mode;
  r.y0 = mp.y0;
  r.nrows = mp.nrows;
  r.ncols = mp.ncols;
  r.step = mp.step;
  r.max_step = mp.max_step;
  r.band_h = mp.band_h;
  r.rank = mp.rank;
  r.world = mp.world;
  r.width = o->width;
  r.height = o->height;
  r.ngroups = p.ngroups;
  r.info = s->fr.info.p;
  r.records = records ? 1 : 0;
  if (records && s->skippable && s->skip_planes.size() <= (size_t)kFrameMaxPlanes) {
    std::vector<bg::SkipPlaneC> pcs;
    if (skip_camera(s->skip_planes, s->mesh_w2o, s->c2w, s->fov, o->width, o->height, o->bias, &r.cam, &pcs)) {
      r.nplanes = (int32_t)pcs.size();
      std::copy(pcs.begin(), pcs.end(), r.planes);
      r.nl = std::min(8, s->nlight);
      for (int l = 0; l < r.nl; ++l) r.have |= s->grid_occ[(size_t)l].g.gu > 0 ? 1u << l : 0u;
      r.grids = s->grids.p;
      r.sat = s->sat_dev.p;
      for (int l = 0; l < 8; ++l) r.sat_off[l] = s->sat_off[l];
    }
  }
  r.split = split ? 1 : 0;
  r.full = s->nlight >= 32 ? ~0u : (1u << s->nlight) - 1u;
  r.lean = s->fr.lean.p;
  r.heavy = s->fr.heavy.p;
  r.ctr = s->fr.ctr.p;
}

// The mesh's camera-ray lists for the launch's pixels, their records
// (records: one-pixel groups) and with split the lean / general lists — the
// call's two build launches (rt_frame.h). *ok = false: no lists for this
// camera (a mesh vertex may lie at or behind the camera plane), the kernels
// traverse the BVH. zero (words, count): the render kernels' queue heads +
// Stats words, zeroed by the first build launch (*zeroed = true).
int frame_build(rt_scene* s, const rt_options* o, const Mapping& mp, const FastParams& p, bool records, bool split,
                unsigned int* zero, int nzero, hipStream_t st, bool* ok, bool* zeroed) {
  *ok = false;
  *zeroed = false;
  if (!s->binnable || s->bin_tris.empty()) return RT_OK;
  FrameLaunch a;
  std::memset(&a, 0, sizeof a);
  if (!pixel_camera(s->mesh_o2w, s->mesh_w2o, s->c2w, s->fov, o->width, o->height, &a.cam)) return RT_OK;
  // every vertex strictly in front of the camera plane (face_pixel_rect's
  // test): the test's left side is convex in the point, so the mesh box's
  // corners bound it
  for (int c = 0; c < 8; ++c) {
    const double q[3] = {(c & 1) ? s->mesh_hi[0] : s->mesh_lo[0], (c & 2) ? s->mesh_hi[1] : s->mesh_lo[1],
                         (c & 4) ? s->mesh_hi[2] : s->mesh_lo[2]};
    double pw[3], pc[3];
    bg::xform_point(s->mesh_o2w, q, pw);
    bg::xform_point(a.cam.w2c, pw, pc);
    if (!(pc[2] < -1e-9 * (1.0 + std::fabs(pc[0]) + std::fabs(pc[1])))) return RT_OK;
  }
  int rc = frame_buffers(s, o->width, o->height, st);
  if (rc) return rc;
  rt_scene::Frame& f = s->fr;
  a.tris = s->bin_dev.p;
  a.nf = (int32_t)s->bin_tris.size();
  a.rows = frame_rows(mp, o->height);
  a.cnt = f.cnt.p;
  a.slots = f.slots.p;
  a.slot_lg = f.slot_lg;
  a.huge = f.huge.p;
  a.parity = (int32_t)(f.calls++ & 1u);
  records_launch(s, o, mp, p, records, split, a.r);
  a.tile_bits = f.tiles.p;
  a.tile_cls = f.status.p;
  static const int diag_b2 = rtmi::diag_env("RTMI_DIAG_B2") ? std::atoi(rtmi::diag_env("RTMI_DIAG_B2")) : 0;
  a.diag = diag_b2;  // diagnostic builds only (probe modes, wrong images)
  a.tiles_x = (mp.ncols + 63) / 64;
  a.ntiles = a.tiles_x * ((mp.nrows + 3) / 4);
  a.zero = zero;
  a.nzero = nzero;
  if ((rc = rtmi_frame_build(&a, st))) {
    // the first launch may have run (its counters non-zero, zeroed only by
    // the second): the next call re-allocates and re-zeroes the buffers
    f.invalidate();
    return fail(RT_E_DEVICE, "frame build launch failed: %s", hipGetErrorString((hipError_t)rc));
  }
  f.listed = true;
  *zeroed = zero != nullptr;
  *ok = true;
  return RT_OK;
}

// Object masks of the launch's rows (k_frame_obj_masks).
int frame_obj_masks(rt_scene* s, const rt_options* o, const Mapping& mp, hipStream_t st, bool* ok) {
  *ok = false;
  ObjMaskLaunch a;
  std::memset(&a, 0, sizeof a);
  static const double kIdentity[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  bg::PixCam pc;
  if (!pixel_camera(kIdentity, kIdentity, s->c2w, s->fov, o->width, o->height, &pc)) return RT_OK;
  int rc = frame_buffers(s, o->width, o->height, st);
  if (rc) return rc;
  a.objs = s->objbox_dev.p;
  a.nobj = s->nobj;
  a.width = o->width;
  a.height = o->height;
  std::memcpy(a.w2c, pc.w2c, sizeof a.w2c);
  a.cam_a = pc.cam_a;
  a.cam_c = pc.cam_c;
  a.margin = kPixelMargin;
  a.rows = frame_rows(mp, o->height);
  a.masks = s->fr.omask.p;
  a.rects = s->fr.orect.p;
  const int e = rtmi_frame_obj_masks(&a, st);
  if (e) return fail(RT_E_DEVICE, "object mask launch failed: %s", hipGetErrorString((hipError_t)e));
  *ok = true;
  return RT_OK;
}

// Every sample offset of the sampler lies in [0, 1) x [0, 1) of its pixel
// (sampling.nim:5-113, renderer.nim:135), the premise of the camera-ray bins
// (rt_bins.h kPixelMargin). A sampler outside this list gets no bins.
bool sampler_in_pixel(int32_t aa_kind) {
  switch (aa_kind) {
    case RT_AA_NONE:                    // the pixel corner: offset 0
    case RT_AA_GRID:                    // (i + 1/2) / m
    case RT_AA_JITTERED:                // (i + u) / m, u in [0, 1)
    case RT_AA_MULTI_JITTERED:          // (i + (j + u) / n) / m
    case RT_AA_CORRELATED_MULTI_JITTERED:
      return true;
    default:
      return false;
  }
}

// The float32 launch's parameters, and this call's camera-dependent data
// built on the device (rt_frame.h) in stream order before the render
// kernels: the mesh's camera-ray lists (>= 16 samples per pixel), the object
// masks, and for one-pixel waves the pixel records — with *split, also the
// lean / general lists of a two-class launch.
// zero / nzero: the render kernels' queue heads + Stats words; a call that
// builds pixel lists zeroes them in its first build launch (*zeroed), else
// the caller clears them.
int fill_fast(rt_scene* s, const rt_options* o, const Mapping& mp, float* fb, FastParams& p, int* blocks,
              rt_scene::Order** measuring, hipStream_t st, bool* split, unsigned int* zero, int nzero, bool* zeroed) {
  std::memset(&p, 0, sizeof p);
  p.objs = s->f32.objs.p;
  p.objx = s->f32.objx.p;
  p.meshes = s->f32.meshes.p;
  p.lights = s->f32.lights.p;
  p.tree = s->f32.tree.p;
  p.normals = s->f32.normals.p;
  p.fb = fb;
  p.partials = s->partials.p;
  p.queue = s->queue.p;
  // camera: origin = C2W * (0,0,0,1) = column 3; dir = C2W * normalize(cx, cy, -1, 0)
  for (int k = 0; k < 3; ++k) {
    p.cam[k] = (float)s->c2w[12 + k];
    p.cam[3 + k] = (float)s->c2w[0 + k];
    p.cam[6 + k] = (float)s->c2w[4 + k];
    p.cam[9 + k] = (float)s->c2w[8 + k];
  }
  const double f = std::tan(s->fov * (3.14159265358979323846 / 180.0) / 2);
  const double r = (double)o->width / (double)o->height;
  p.cam_a = (float)(2.0 * r * f / (double)o->width);  // cx = ((2 x r)/w - r) f = (x - w/2) 2rf/w
  p.cam_b = (float)(0.5 * (double)o->width);
  p.cam_c = (float)(2.0 * f / (double)o->height);     // cy = (1 - 2y/h) f = (h/2 - y) 2f/h
  p.cam_d = (float)(0.5 * (double)o->height);
  for (int k = 0; k < 3; ++k) p.bg[k] = (float)s->bg[k];
  p.bias = (float)o->bias;
  const int m = o->aa_kind != RT_AA_NONE ? o->grid_size : 1;
  const int spp = m * m;
  p.inv_len = (float)(1.0 / (double)spp);
  p.sample_step = (float)(1.0 / (double)m);
  p.sample_off = (float)(1.0 / (double)m * 0.5);
  p.log2_grid_m = -1;
  for (int k = 0; k <= 12; ++k)
    if (m == (1 << k)) p.log2_grid_m = k;
  p.nobj = s->nobj;
  p.nlight = s->nlight;
  p.has_point_light = s->has_point_light;
  p.seed = o->seed;
  p.width = o->width;
  p.height = o->height;
  p.aa_kind = o->aa_kind;
  p.grid_m = m;
  p.spp = spp;
  p.max_depth = o->max_ray_depth;
  p.flags = (int32_t)o->flags;
  p.shadow_mesh = s->shadow_mesh;
  p.mode = mp.mode;
  p.y0 = mp.y0;
  p.nrows = mp.nrows;
  p.ncols = mp.ncols;
  p.step = mp.step;
  p.max_step = mp.max_step;
  p.band_h = mp.band_h;
  p.rank = mp.rank;
  p.world = mp.world;
  const Plan pl = plan_mapping(s, o, mp, spp);
  p.lanes_per_px = pl.L;
  p.log2_lanes = pl.log2L;
  p.tile_x = pl.tx;
  p.tile_y = pl.ty;
  p.log2_tile_x = 0;
  while ((1 << p.log2_tile_x) < pl.tx) ++p.log2_tile_x;
  p.inv_band_h = mp.band_h > 0 ? (float)(1.0 / (double)mp.band_h) : 0.0f;
  p.tiles_x = pl.tiles_x;
  p.ngroups = pl.ngroups;
  p.iters = (spp + pl.L - 1) / pl.L;
  {  // g / tiles_x by multiply-shift: m = floor(2^(31+s) / d) + 1, s = ceil(log2 d), exact for g < 2^31
    const uint64_t d = (uint64_t)std::max(1, pl.tiles_x);
    int sh = 0;
    while ((1ull << sh) < d) ++sh;
    p.tx_shift = 31 + sh;
    p.tx_magic = (uint32_t)((1ull << (31 + sh)) / d + 1ull);
  }
  {  // the 32-bit wave counters stay in registers across work items and are
     // added to the 64-bit totals before any can wrap: per item at most
     // 64 lanes x iters samples x levels x (1 + lights) traces x objects hits
    const uint64_t levels = s->any_reflective ? (uint64_t)std::min(kMaxShadeLevels, std::max(1, o->max_ray_depth + 1)) : 1ull;
    const uint64_t per_item = 64ull * (uint64_t)p.iters * levels * (1ull + (uint64_t)s->nlight) *
                              (uint64_t)std::max(1, s->nobj);
    // diagnostic builds with wider counters (RTMI_DIAG_LANES): RTMI_STAT_FLUSH=1 flushes every item
    static const int flush_env = rtmi::diag_env("RTMI_STAT_FLUSH") ? std::atoi(rtmi::diag_env("RTMI_STAT_FLUSH")) : 0;
    p.stat_flush = (o->flags & RT_FLAG_COUNT_TRAVERSAL) ? 1
                   : flush_env > 0 ? flush_env
                                   : (int32_t)std::min<uint64_t>(1u << 20, std::max<uint64_t>(1, 0xFFFFFFFFull / per_item));
  }
  // binned searches (rt_bins.h): camera rays when a wave spans at most 4
  // pixels (>= 16 samples per pixel), shadow rays to distant lights
  // the shadow-ray records: on every path (binned or not), so every path
  // tests a distant light's shadow rays with the same arithmetic
  if (s->lrec.p) {
    p.lrec_base = (uint64_t)(uintptr_t)s->lrec.p - (uint64_t)s->num_nodes * sizeof(TriFast);
    p.lrec_stride = s->lrec_ntri * (int64_t)sizeof(LTri);
    p.lrec_mask = s->lrec_mask;
    p.grid_rec = s->grec.p;
  }
  const bool binning = !(o->flags & RT_FLAG_NO_BINNING);
  if (binning) {
    if (s->has_grids) {
      p.grids = s->grids.p;
      p.grid_off = s->grid_off.p;
      p.grid_ent = s->grid_ent.p;
    }
    if (s->has_obj_grids) {
      p.obj_grids = s->obj_grids.p;
      p.obj_grid_mask = s->obj_grid_mask.p;
      p.obj_off_grid = s->obj_off_grid;
    }
  }
  // one work item per dequeue: per-pixel cost varies ~10x (sky vs bunny +
  // shadows), so coarser chunks leave an expensive tail in every launch
  // (C3 whole frame: 4 groups per dequeue 9.79 ms, 1 9.49 ms; 2-way bands:
  // 5.22 vs 4.69 ms per half). With 8 sharded heads the dequeue rate stays
  // far below the ~90/us a head sustains.
  p.shards = std::min(kQueueShards, pl.blocks);
  const OrderUse ou = group_order(s, o, mp, p, pl.blocks);
  p.order = ou.order;
  p.cost = ou.cost;
  *measuring = ou.entry;
  *blocks = pl.blocks;
  *split = false;
  *zeroed = false;
  if (!binning || pl.L < 16 || !sampler_in_pixel(o->aa_kind)) return RT_OK;
  // this call's camera-dependent data (nothing of it is kept from earlier calls)
  int rc;
  bool lists = false, masks = false;
  // two-class launch (one pixel per wave): the lean pixels — no camera ray
  // can hit the mesh, every light a distant light whose shadow rays from the
  // pixel provably miss it, no reflection — get a kernel of their own; not
  // for the measuring launch of a launch order or instrumented launches
  static const char* cost_dump = rtmi::diag_env("RTMI_COST_DUMP");
  const unsigned sub = f32_subset(s, o);
  const bool want_split = !(o->flags & (RT_FLAG_NO_SPLIT | RT_FLAG_COUNT_TRAVERSAL)) && !p.cost && !cost_dump &&
                          s->nlight <= 8 && rtmi_lean_f32_blocks_per_cu(sub, f32_table_lds(s, o)) > 0;
  const bool records = pl.L == 64;  // one-pixel groups: records (+ the split)
  *split = records && want_split && !p.order;
  // the build on the scene's build stream after the call two back (the last
  // user of this buffer set), joined into the caller's stream before the
  // render kernels: it overlaps the previous call's render
  hipStream_t bs = st;
  if (s->pipe) {
    bs = s->bstream;
    if (s->fr.used_rec) HIP_TRY(hipStreamWaitEvent(bs, s->fr.used, 0));
  }
  auto join = [&]() -> int {
    if (bs != st) {
      HIP_TRY(hipEventRecord(s->fr.built, bs));
      HIP_TRY(hipStreamWaitEvent(st, s->fr.built, 0));
    }
    return RT_OK;
  };
  if ((rc = frame_build(s, o, mp, p, records, *split, zero, nzero, bs, &lists, zeroed))) {
    join();
    return rc;
  }
  if (lists) {
    p.pix_slots = s->fr.slots.p;
    p.pix_cnt = s->fr.info.p;
    p.slot_lg = s->fr.slot_lg;
    if (records) p.pix_info = s->fr.info.p;
  } else {
    *split = false;
  }
  if (s->objbins) {
    if ((rc = frame_obj_masks(s, o, mp, bs, &masks))) {
      join();
      return rc;
    }
    if (masks) p.obj_pix = s->fr.omask.p;
  }
  return join();
}

template <class R>
void fill_params(rt_scene* s, const PrecisionData<R>& pd, const rt_options* o, const Mapping& mp, float* fb,
                 RenderParams<R>& p, int* blocks) {
  std::memset(&p, 0, sizeof p);
  p.objects = pd.objects.p;
  p.lights = pd.lights.p;
  p.meshes = pd.meshes.p;
  p.nodes = s->nodes.p;
  p.tris = pd.tris.p;
  p.normals = pd.normals.p;
  p.fb = fb;
  p.partials = s->partials.p;
  for (int k = 0; k < 16; ++k) p.c2w[k] = (R)s->c2w[k];
  for (int k = 0; k < 3; ++k) p.bg[k] = (R)s->bg[k];
  // castPrimaryRay constants (renderer.nim:36-38), float64 on the host
  p.f = (R)std::tan(s->fov * (3.14159265358979323846 / 180.0) / 2);
  p.aspect = (R)((double)o->width / (double)o->height);
  p.bias = (R)o->bias;
  const int m = o->aa_kind != RT_AA_NONE ? o->grid_size : 1;
  const int spp = m * m;
  p.inv_len = (R)(1.0 / (double)spp);
  const double xs = 1.0 / (double)m;  // grid(): xs = 1/n, ys = 1/m (m = n)
  p.sample_step = (R)xs;
  p.sample_off = (R)(xs * 0.5);
  p.nobj = s->nobj;
  p.nlight = s->nlight;
  p.width = o->width;
  p.height = o->height;
  p.aa_kind = o->aa_kind;
  p.grid_m = m;
  p.spp = spp;
  p.max_depth = o->max_ray_depth;
  p.flags = (int32_t)o->flags;
  p.shadow_mesh = s->shadow_mesh;
  p.lean_plane = -1;
  p.seed = o->seed;
  p.sample_scratch = nullptr;
  p.max_iters = (int32_t)std::min<int64_t>(INT32_MAX, 2 * s->num_nodes + 16);
  p.mode = mp.mode;
  p.y0 = mp.y0;
  p.nrows = mp.nrows;
  p.ncols = mp.ncols;
  p.step = mp.step;
  p.max_step = mp.max_step;
  p.band_h = mp.band_h;
  p.rank = mp.rank;
  p.world = mp.world;
  // lanes per pixel: float64 parity mode keeps the reference's sequential
  // sample sum (one lane per pixel); float32 spreads samples over lanes.
  int L = 1;
  if (o->precision == RT_FP32) {
    while (L * 2 <= std::min(spp, 64)) L *= 2;
  }
  const int P = 64 / L;
  int tx = 1, ty = 1;
  switch (P) {
    case 64: tx = 8; ty = 8; break;
    case 32: tx = 8; ty = 4; break;
    case 16: tx = 4; ty = 4; break;
    case 8: tx = 4; ty = 2; break;
    case 4: tx = 2; ty = 2; break;
    case 2: tx = 2; ty = 1; break;
    default: tx = 1; ty = 1; break;
  }
  p.lanes_per_px = L;
  p.tile_x = tx;
  p.tile_y = ty;
  p.tiles_x = (mp.ncols + tx - 1) / tx;
  const long long tiles_y = (mp.nrows + ty - 1) / ty;
  p.ngroups = (long long)p.tiles_x * tiles_y;
  const long long want = (p.ngroups + 3) / 4;
  long long cap = s->max_waves / 4;
  if (o->aa_kind >= RT_AA_JITTERED) {  // per-lane sample tables: keep the scratch <= 256 MB
    const long long per_block = 256LL * 2 * spp * (long long)sizeof(R);
    cap = std::min(cap, std::max(1LL, (256LL << 20) / per_block));
  }
  *blocks = (int)std::max(1LL, std::min<long long>(want, cap));
}

// k_render_lean1 (rt_fast.h) renders the lean pixels when the scene's only
// analytic object is one plane and every transform a translation (the
// mesh + plane feature subset, nothing else), with one or two distant lights,
// and akGrid sampling with m | 64 whose samples fill whole 4-sample batches
// of every lane (spp a multiple of 256): every sample is valid and a lane's
// samples share one column. Off with RT_FLAG_NO_LEAN1. The general pixels of
// the same launches go to k_render_gen1 (off with RT_FLAG_NO_GEN1).
// Whether a one-plane two-class launch runs as one merged kernel
// (k_render_mix1). RTMI_MIX=0/1 forces it (diagnostic A/B); by default:
// always.
bool mix_policy() {
  static const int force = rtmi::diag_env("RTMI_MIX") ? std::atoi(rtmi::diag_env("RTMI_MIX")) : -1;
  return force != 0;
}

bool lean1_ok(const rt_scene* s, const rt_options* o, const FastParams& p, unsigned sub) {
  return sub == SUB_MESH && p.nobj == 2 && p.shadow_mesh >= 0 &&
         (p.nlight == 1 || p.nlight == 2) && !p.has_point_light && p.aa_kind == RT_AA_GRID &&
         p.log2_grid_m >= 0 && p.log2_grid_m <= 6 && p.lanes_per_px == 64 && p.spp % 256 == 0 &&
         p.iters * 64 == p.spp && p.iters % 4 == 0 && s->nobj == 2;
}

// zero / nzero: the queue heads and / or Stats words every call clears
// before its render kernels (a float32 call that builds pixel lists clears
// them in its first build launch: one launch fewer).
int launch(rt_scene* s, const rt_options* o, const Mapping& mp, float* d_out, hipStream_t st, bool reduce,
           unsigned int* zero, int nzero) {
  int blocks = 1;
  auto clear = [&]() -> int {
    if (nzero > 0) HIP_TRY(hipMemsetAsync(zero, 0, (size_t)nzero * sizeof(unsigned int), st));
    return RT_OK;
  };
  // what rt_scene_last_split / _last_batch report describes THIS call, even
  // when it returns early or runs the float64 kernel
  s->fr.counted = false;
  s->fr.listed = false;
  s->pending_reduce = 0;
  s->last_lean = 0;
  s->last_lean_kind = 0;
  s->last_general = 0;
  s->last_batched = 0;
  if (o->precision == RT_FP64) {
    if (int rc = clear()) return rc;
    RenderParams<double> p;
    fill_params<double>(s, s->f64, o, mp, d_out, p, &blocks);
    s->last_general = p.ngroups;
    if (p.ngroups == 0) return RT_OK;
    if (p.aa_kind >= RT_AA_JITTERED) {
      const size_t need = (size_t)blocks * 256 * 2 * (size_t)p.spp;
      if (s->f64_tables.n < need) {
        HIP_TRY(hipStreamSynchronize(st));  // an earlier launch may still use the old buffer
        int rc = s->f64_tables.alloc(need);
        if (rc) return rc;
      }
      p.sample_scratch = s->f64_tables.p;
    }
    s->last_lean = 0;
    s->last_lean_kind = 0;
    s->last_general = p.ngroups;
    s->last_batched = 0;
    // this call's pixel records (the float32 path's build, one launch set):
    // a pixel whose camera rays provably miss the mesh skips their traversal,
    // and its shadow rays to the lights its skip bits clear skip theirs —
    // the same answers (the traversal would find no face), so frames and
    // Stats stay bit-exact (tests/test_gpu_parity.py)
    const bool binning = !(o->flags & (RT_FLAG_NO_BINNING | RT_FLAG_COUNT_TRAVERSAL));
    bool lists = false;
    if (binning && sampler_in_pixel(o->aa_kind) && s->skippable) {
      FastParams pf;
      std::memset(&pf, 0, sizeof pf);
      bool zeroed = false;
      if (int rc = frame_build(s, o, mp, pf, true, false, nullptr, 0, st, &lists, &zeroed)) return rc;
      if (lists) p.pix_info = s->fr.info.p;
    }
    // one pixel per wave (k_render_px64): akGrid with >= 64 samples per
    // pixel; the camera rays search this call's pixel lists, the shadow rays
    // to distant lights the scene's light grids (rt_device.h mesh_lists)
    const int px64 = o->aa_kind == RT_AA_GRID && p.spp >= 64 && !(o->flags & (RT_FLAG_F64_PER_LANE | RT_FLAG_COUNT_TRAVERSAL))
                         ? (s->any_reflective && o->max_ray_depth >= 1 ? 2 : 1)
                         : 0;
    if (px64) {
      if (lists) {
        p.pix_slots = s->fr.slots.p;
        p.slot_lg = s->fr.slot_lg;
        p.lean_plane = s->lean64_plane;
      }
      if (binning && s->has_grids) {
        p.grids = s->grids.p;
        p.grid_off = s->grid_off.p;
        p.grid_ent = s->grid_ent.p;
        if (!s->sh64_ready && s->shadow_mesh >= 0) {
          if (int rc = s->sh64.alloc(s->grid_ent.n)) return rc;
          for (int li = 0; li < s->nlight && li < (int)s->grid_host.size(); ++li) {
            const LightGridHost& lg = s->grid_host[(size_t)li];
            if (lg.g.gu <= 0 || lg.ent.empty()) continue;
            const int e = rtmi_build_sh64(s->f64.objects.p, s->shadow_mesh, s->f64.lights.p, li,
                                          s->grid_ent.p + lg.g.ent_base, (int)lg.ent.size(), s->f64.tris.p,
                                          (int32_t)s->num_nodes, s->sh64.p + lg.g.ent_base, st);
            if (e) return fail(RT_E_DEVICE, "shadow record build failed: %s", hipGetErrorString((hipError_t)e));
          }
          s->sh64_ready = true;
        }
        if (s->sh64_ready) p.sh64 = s->sh64.p;
      }
      p.tri_rec0 = (int32_t)s->num_nodes;
      const long long nbatch = ((long long)mp.nrows * mp.ncols + rtmi_px64_batch() - 1) / rtmi_px64_batch();
      const long long resident = (long long)std::max(1, rtmi_px64_blocks_per_cu(px64)) * s->num_cus;
      blocks = (int)std::max(1LL, std::min({(nbatch + 3) / 4, resident, (long long)s->max_waves / 4}));
    }
    if (o->flags & RT_FLAG_TIMING) HIP_TRY(hipEventRecord(s->tev[1], st));  // after the per-call build
    const int e = rtmi_launch_render_f64(&p, blocks, px64, st);
    if (e) return fail(RT_E_DEVICE, "render kernel launch failed: %s", hipGetErrorString((hipError_t)e));
  } else {
    FastParams p;
    rt_scene::Order* measuring = nullptr;
    bool split = false, zeroed = false;
    if (mp.nrows == 0 || mp.ncols == 0) return clear();
    int rc = fill_fast(s, o, mp, d_out, p, &blocks, &measuring, st, &split, zero, nzero, &zeroed);
    if (rc) return rc;
    if (!zeroed && (rc = clear())) return rc;
    if (o->flags & RT_FLAG_TIMING) HIP_TRY(hipEventRecord(s->tev[1], st));
    s->last_general = p.ngroups;
    if (p.ngroups == 0) return RT_OK;
    // diagnostic (tools/cost_map.py): RTMI_COST_DUMP=<file> records every
    // pixel group's duration (s_memtime cycles) of this launch into <file>
    static const char* cost_dump = rtmi::diag_env("RTMI_COST_DUMP");
    DevBuf<unsigned> dbg_cost;
    if (cost_dump && !measuring && !p.cost) {
      if (dbg_cost.alloc((size_t)p.ngroups) == RT_OK) p.cost = dbg_cost.p;
    }
    s->fr.counted = split;
    if (split) {  // two-class launch: the general kernel on its list, then the lean kernel on its own
      // the lists and their entry counts come from this call's k_frame_build2
      // (the host never reads them: grids and items are sized for the launch's
      // groups, the kernels stop at the device counts)
      int32_t* const n_heavy = s->fr.ctr.p + FC_HEAVY;
      int32_t* const n_lean = s->fr.ctr.p + FC_LEAN;
      const size_t shmem = f32_table_lds(s, o);
      const unsigned sub = f32_subset(s, o);
      FastParams ph = p, pl = p;
      // the general pixels: the batched kernel (k_render_gen) for scenes of
      // one mesh object with distant lights only, no reflection (the lean
      // kernel's subsets) when both camera lists and light grids exist
      const int gbpc = (o->flags & RT_FLAG_NO_BATCH) || p.shadow_mesh < 0 || !p.pix_slots || !p.grids ||
                               p.has_point_light
                           ? 0
                           : rtmi_gen_f32_blocks_per_cu(sub, shmem);
      const bool gen = gbpc > 0;
      const bool one_plane = lean1_ok(s, o, p, sub);
      const bool gen1 = gen && one_plane && !(o->flags & RT_FLAG_NO_GEN1);
      const long long hcap =
          gen ? std::min<long long>((long long)(gen1 ? rtmi_gen1_f32_blocks_per_cu(p.nlight) : gbpc) * s->num_cus, blocks)
              : blocks;
      // diagnostic: RTMI_GEN_WAVES_CAP / RTMI_LEAN_WAVES_CAP = resident waves per SIMD each kernel may take
      static const int gen_cap = rtmi::diag_env("RTMI_GEN_WAVES_CAP") ? std::atoi(rtmi::diag_env("RTMI_GEN_WAVES_CAP")) : 0;
      static const int lean_cap = rtmi::diag_env("RTMI_LEAN_WAVES_CAP") ? std::atoi(rtmi::diag_env("RTMI_LEAN_WAVES_CAP")) : 0;
      const long long hcap2 = gen_cap > 0 ? std::min<long long>(hcap, (long long)gen_cap * s->num_cus) : hcap;
      const int hb = (int)std::max(1LL, std::min<long long>(hcap2, ((long long)p.ngroups + 3) / 4));
      ph.order = s->fr.heavy.p;
      ph.ngroups = p.ngroups;
      ph.list_n = n_heavy;
      ph.shards = std::min(kQueueShards, hb);
      const bool lean1 = one_plane && !(o->flags & RT_FLAG_NO_LEAN1);
      // work items: runs of kLeanRun pixels (k_render_lean, k_render_lean1),
      // 64 / lp pixels (k_render_lean1q, lp lanes per pixel): 16 per item
      // unless the launch's groups make fewer items than resident waves (a
      // short launch, e.g. a scanline), then 4. (Round 3 switched below 8
      // items per wave; a rank's bands at N = 8 — 2 per wave — render faster
      // at 16 pixels per item in a back-to-back loop: 0.1605 -> 0.1539 ms,
      // N = 4 0.278 -> 0.265 ms, profiles/r4/ab/r4t_*)
      const long long lwaves4 =
          4LL * std::min<long long>((long long)rtmi_lean1_f32_blocks_per_cu(p.nlight, 4) * s->num_cus, s->max_waves / 4);
      static const int lp_env = rtmi::diag_env("RTMI_LEAN_LP") ? std::atoi(rtmi::diag_env("RTMI_LEAN_LP")) : 0;  // diagnostic: 4 / 16
      const int lp = !(lean1 && rtmi_lean1_quads())
                         ? 64
                         : (lp_env == 4 || lp_env == 16 ? lp_env : ((long long)(p.ngroups + 15) / 16 >= lwaves4 ? 4 : 16));
      const long long lcap =
          (long long)(lean1 ? rtmi_lean1_f32_blocks_per_cu(p.nlight, lp) : rtmi_lean_f32_blocks_per_cu(sub, shmem)) *
          s->num_cus;
      const int lrun = lp == 64 ? kLeanRun : 64 / lp;
      const int lruns = (p.ngroups + lrun - 1) / lrun;  // at most: the kernels stop at the device count
      const long long lcap2 = lean_cap > 0 ? std::min<long long>(lcap, (long long)lean_cap * s->num_cus) : lcap;
      const int lb = (int)std::max(1LL, std::min<long long>(std::min<long long>(lcap2, s->max_waves / 4),
                                                            ((long long)lruns + 3) / 4));
      pl.order = s->fr.lean.p;
      pl.ngroups = lruns;
      pl.list_n = n_lean;
      pl.stat_flush = std::max(1, p.stat_flush / lrun);
      pl.shards = std::min(kQueueShards, lb);
      pl.queue = s->queue.p + (size_t)kQueueShards * kQueueStride;
      pl.partials = s->partials.p + (size_t)hb * 4 * kStatSlots;
      // one-plane launches: both lists in one kernel (k_render_mix1: the
      // general items first, then the lean ones) — one ramp and one tail
      const bool mix = gen1 && lean1 && lp != 64 && !(o->flags & RT_FLAG_NO_MIX) && mix_policy();
      if (mix) {
        FastParams pm = ph;
        pm.order2 = pl.order;
        pm.ngroups2 = pl.ngroups;
        pm.list_n2 = n_lean;
        pm.stat_flush = std::min(ph.stat_flush, pl.stat_flush);
        const long long mcap = (long long)rtmi_mix1_f32_blocks_per_cu(p.nlight, lp) * s->num_cus;
        const int mb = (int)std::max(1LL, std::min<long long>(std::min<long long>(mcap, blocks),
                                                              ((long long)p.ngroups + lruns + 3) / 4));
        static const int shard_cap = rtmi::diag_env("RTMI_SHARDS") ? std::atoi(rtmi::diag_env("RTMI_SHARDS")) : 0;  // diagnostic
        pm.shards = std::min(shard_cap > 0 ? std::min(shard_cap, kQueueShards) : kQueueShards, mb);
        pm.shards2 = pm.shards;
        // diagnostic (RTMI_PIPE_GRID=<percent>): a pipelined call's grid capped,
        // leaving CU slots to the next call's build
        static const int pipe_grid = rtmi::diag_env("RTMI_PIPE_GRID") ? std::atoi(rtmi::diag_env("RTMI_PIPE_GRID")) : 0;
        const int mbl = s->pipe && pipe_grid > 0 ? std::max(1, (int)((long long)mb * pipe_grid / 100)) : mb;
        const int e = rtmi_launch_mix1_f32(&pm, p.nlight, lp, mbl, st);
        if (e) return fail(RT_E_DEVICE, "render kernel launch failed: %s", hipGetErrorString((hipError_t)e));
        blocks = mb;
        s->last_lean_kind = 3 | (3 << 2) | (lp << 8);
        s->last_batched = -1;  // = the general list (device count)
        goto launched;
      }
      // general kernel first on the caller's stream, the lean kernel on
      // the scene's aux stream (forked after the caller's earlier work,
      // joined before its later work)
      static const bool serial = rtmi::diag_env("RTMI_SPLIT_SERIAL") != nullptr;  // diagnostic: one stream
      hipStream_t sl = serial ? st : s->aux;
      if (!serial) {
        HIP_TRY(hipEventRecord(s->fork, st));
        HIP_TRY(hipStreamWaitEvent(s->aux, s->fork, 0));
      }
      static const bool lean_first = rtmi::diag_env("RTMI_LEAN_FIRST") != nullptr;  // diagnostic
      auto launch_lean = [&]() {
        return lean1 ? rtmi_launch_lean1_f32(&pl, p.nlight, lp, lb, sl) : rtmi_launch_lean_f32(&pl, sub, lb, shmem, sl);
      };
      int e = lean_first ? launch_lean() : 0;
      if (!e)
        e = gen1  ? rtmi_launch_gen1_f32(&ph, p.nlight, hb, st)
            : gen ? rtmi_launch_gen_f32(&ph, sub, hb, shmem, st)
                  : rtmi_launch_render_f32(&ph, sub, hb, shmem, st);
      if (!e && !lean_first) e = launch_lean();
      if (e) return fail(RT_E_DEVICE, "render kernel launch failed: %s", hipGetErrorString((hipError_t)e));
      if (!serial) {
        HIP_TRY(hipEventRecord(s->join, s->aux));
        HIP_TRY(hipStreamWaitEvent(st, s->join, 0));
      }
      blocks = hb + lb;
      s->last_lean_kind = (lean1 ? 2 : 1) | ((gen1 ? 2 : gen ? 1 : 0) << 2) | (lp << 8);
      s->last_batched = gen ? -1 : 0;
    } else {
      s->last_lean = 0;
      s->last_lean_kind = 0;
      s->last_general = p.ngroups;
      s->last_batched = 0;
      const unsigned sub = f32_subset(s, o);
      const size_t shmem = f32_table_lds(s, o);
      // RT_FLAG_COMPACT, reflective scenes: reflected rays compacted per wave
      // (k_render_wave); not for an instrumented launch or a progressive
      // pass that fills step x step blocks (its pixels' sums are stored
      // more than once)
      const long long span = (long long)mp.nrows * o->width;
      const int wbpc = (sub & SUB_REFLECT) && (o->flags & RT_FLAG_COMPACT) && !(o->flags & RT_FLAG_COUNT_TRAVERSAL) &&
                               !(mp.mode == 0 && mp.step > 1) && span < (1ll << 27)
                           ? rtmi_wave_f32_blocks_per_cu(sub, shmem)
                           : 0;
      if (wbpc > 0) {
        const int wb = (int)std::max(1LL, std::min<long long>(std::min<long long>((long long)wbpc * s->num_cus,
                                                                                  s->max_waves / 4),
                                                              ((long long)p.ngroups + 3) / 4));
        const size_t qfl = (size_t)wb * 4 * kReflQueue * kReflFields;
        const size_t nsec = (size_t)span * 3;
        if (s->refl_queue.n < qfl || s->refl_sec.n < nsec) {
          HIP_TRY(hipStreamSynchronize(st));  // an earlier launch may still use the old buffers
          int rc2 = s->refl_queue.n < qfl ? s->refl_queue.alloc(qfl) : RT_OK;
          if (!rc2 && s->refl_sec.n < nsec) rc2 = s->refl_sec.alloc(nsec);
          if (rc2) return rc2;
        }
        HIP_TRY(hipMemsetAsync(s->refl_sec.p, 0, nsec * sizeof(long long), st));
        p.rq = s->refl_queue.p;
        p.sec = s->refl_sec.p;
        p.sec_base = mp.mode == 0 ? (int64_t)mp.y0 * o->width : 0;
        p.shards = std::min(kQueueShards, wb);
        int e = rtmi_launch_wave_f32(&p, sub, wb, shmem, st);
        if (!e)
          e = rtmi_launch_sec_add(d_out + (size_t)p.sec_base * 3, p.sec, nsec, o->aa_kind != RT_AA_NONE ? p.inv_len : 1.0f,
                                  s->num_cus, st);
        if (e) return fail(RT_E_DEVICE, "render kernel launch failed: %s", hipGetErrorString((hipError_t)e));
        blocks = wb;
        s->last_lean_kind = 16;
      } else {
        const int e = rtmi_launch_render_f32(&p, sub, blocks, shmem, st);
        if (e) return fail(RT_E_DEVICE, "render kernel launch failed: %s", hipGetErrorString((hipError_t)e));
      }
    }
  launched:
    if (measuring) HIP_TRY(hipEventRecord(measuring->measured, st));
    if (dbg_cost.p) {
      std::vector<unsigned> c((size_t)p.ngroups);
      HIP_TRY(hipStreamSynchronize(st));
      HIP_TRY(hipMemcpy(c.data(), dbg_cost.p, c.size() * sizeof(unsigned), hipMemcpyDeviceToHost));
      dbg_cost.release();
      if (FILE* f = std::fopen(cost_dump, "wb")) {
        std::fwrite(c.data(), sizeof(unsigned), c.size(), f);
        std::fclose(f);
      }
    }
  }
  // the per-wave rows are reduced when the Stats are read (flush_reduce)
  if (reduce) s->pending_reduce = blocks * 4;
  return RT_OK;
}

// The last call's Stats rows into acc(), on stream st (ordered after the
// call): at the end of a call whose caller reads its Stats, else by the
// first rt_scene_last_stats / _last_counters (the scene mutex is held; a
// later call replaces the rows and the pending count).
int flush_reduce(rt_scene* s, hipStream_t st) {
  if (s->pending_reduce <= 0) return RT_OK;
  const int e = rtmi_launch_reduce_stats(s->partials.p, s->pending_reduce, s->acc(), st);
  s->pending_reduce = 0;
  if (e) return fail(RT_E_DEVICE, "stats reduction launch failed: %s", hipGetErrorString((hipError_t)e));
  return RT_OK;
}

int read_stats(rt_scene* s, hipStream_t st, rt_stats* out) {
  unsigned long long h[kStatSlots];
  HIP_TRY(hipMemcpyAsync(h, s->acc(), sizeof h, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  out->num_primary_rays = h[STAT_PRIMARY];
  // renderer.nim:54-56 counts one test per object per trace call, and every
  // trace call is a primary, shadow or reflection ray: the float32 kernel
  // leaves the slot at 0 and the count is derived; the float64 kernel still
  // counts it, which is checked here.
  const unsigned long long rays = h[STAT_PRIMARY] + h[STAT_SHADOW] + h[STAT_REFL];
  const unsigned long long tests = (unsigned long long)s->nobj * rays;
#if !(defined(RTMI_DIAG) && defined(RTMI_PX64_ONLY))  // that diagnostic skips samples on purpose
  if (h[STAT_TESTS] != 0 && h[STAT_TESTS] != tests)
    return fail(RT_E_DEVICE, "inconsistent intersection-test count (%llu vs %llu)", h[STAT_TESTS], tests);
#endif
  out->num_intersection_tests = tests;
  out->num_intersection_hits = h[STAT_HITS];
  out->num_shadow_rays = h[STAT_SHADOW];
  out->num_reflection_rays = h[STAT_REFL];
  s->last_fallback = (int64_t)h[STAT_GEN_FALLBACK];
  return RT_OK;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    prev = device_of_current();
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// Common device-side body: order after the previous call, clear the
// counters, launch, record completion. With RT_FLAG_NO_STATS (and no `out`,
// no traversal counting) the call's Stats are not reduced: it launches its
// render kernels and nothing else, and rt_scene_last_stats reports that.
int render_device(rt_scene* s, const rt_options* o, const Mapping& mp, float* d_out, hipStream_t st,
                  rt_stats* out, bool need_stats = false) {
  const bool reduce = need_stats || out || !(o->flags & RT_FLAG_NO_STATS) || (o->flags & RT_FLAG_COUNT_TRAVERSAL);
  s->stats_kept = reduce;
  // after the scene's previous call (a call on that call's own stream is
  // already ordered after it: no wait packet)
  if (st != s->done_stream) HIP_TRY(hipStreamWaitEvent(st, s->done, 0));
  s->timed = (o->flags & RT_FLAG_TIMING) != 0;
  s->pipe = o->precision == RT_FP32 &&
            (s->pipe_mode == 1 ||
             (s->pipe_mode < 0 && 3LL * mp.nrows * mp.ncols <= (long long)o->width * (long long)o->height));
  if (s->pipe) {  // the other buffer set (the last call's stays intact for its readers until the next call)
    std::swap(s->fr, s->fr2);
    std::swap(s->queue, s->queue2);
  }
  if (s->timed) {  // (tev[1] again before the render kernels; here for launches with nothing to render)
    HIP_TRY(hipEventRecord(s->tev[0], st));
    HIP_TRY(hipEventRecord(s->tev[1], st));
  }
  // one fill: the queue heads (float32) and / or the Stats accumulator behind them
  const size_t q0 = o->precision == RT_FP32 ? 0 : rt_scene::kQueueWords;
  const size_t q1 = rt_scene::kQueueWords + (reduce ? 2 * (size_t)kStatSlots : 0);
  int rc = launch(s, o, mp, d_out, st, reduce, s->queue.p + q0, (int)(q1 - q0));
  if (rc) return rc;
  if ((out || need_stats || (o->flags & RT_FLAG_COUNT_TRAVERSAL)) && (rc = flush_reduce(s, st))) return rc;
  if (s->timed) HIP_TRY(hipEventRecord(s->tev[2], st));
  // one event per call: the set's `used` is also the scene's `done`
  HIP_TRY(hipEventRecord(s->fr.used, st));
  s->fr.used_rec = true;
  s->done = s->fr.used;
  s->done_stream = st;
  if (out) return read_stats(s, st, out);
  return RT_OK;
}

int lines_mapping(const rt_options* o, int32_t y0, int32_t y1, int32_t step, int32_t max_step, Mapping* mp) {
  if (!is_pow2(step) || !is_pow2(max_step) || max_step < step)
    return fail(RT_E_INVALID, "step %d / maxStep %d must be powers of two with maxStep >= step", step, max_step);
  if (y0 < 0 || y1 > o->height || y0 > y1) return fail(RT_E_INVALID, "rows [%d, %d) outside [0, %d)", y0, y1, o->height);
  mp->mode = 0;
  mp->y0 = y0;
  mp->nrows = (y1 - y0 + step - 1) / step;
  mp->ncols = (o->width + step - 1) / step;
  mp->step = step;
  mp->max_step = max_step;
  mp->band_h = 1;
  mp->rank = 0;
  mp->world = 1;
  return RT_OK;
}

}  // namespace

extern "C" int rt_render_lines_device(rt_scene* s, const rt_options* o, float* d_fb, int32_t y0, int32_t y1,
                                      int32_t step, int32_t max_step, void* stream, rt_stats* out) {
  if (!s || !d_fb) return fail(RT_E_INVALID, "null argument");
  int rc = check_options(s, o);
  if (rc) return rc;
  Mapping mp;
  if ((rc = lines_mapping(o, y0, y1, step, max_step, &mp))) return rc;
  std::lock_guard<std::mutex> lk(s->mu);
  DeviceGuard g(s->device);
  return render_device(s, o, mp, d_fb, (hipStream_t)stream, out);
}

extern "C" int rt_render_lines(rt_scene* s, const rt_options* o, float* fb, int32_t fb_w, int32_t fb_h, int32_t y0,
                               int32_t y1, int32_t step, int32_t max_step, rt_stats* out) {
  if (!s || !fb) return fail(RT_E_INVALID, "null argument");
  int rc = check_options(s, o);
  if (rc) return rc;
  if (fb_w != o->width || fb_h != o->height)
    return fail(RT_E_INVALID, "framebuffer %dx%d does not match options %dx%d", fb_w, fb_h, o->width, o->height);
  Mapping mp;
  if ((rc = lines_mapping(o, y0, y1, step, max_step, &mp))) return rc;
  rt_stats local{};
  if (mp.nrows == 0) {
    if (out) *out = local;
    return RT_OK;
  }
  std::lock_guard<std::mutex> lk(s->mu);
  DeviceGuard g(s->device);
  const size_t need = (size_t)o->width * o->height * 3;
  if (s->fb_scratch.n < need && (rc = s->fb_scratch.alloc(need))) return rc;
  // rows the call may write: renderLine fills step x step blocks below y
  const int32_t last_y = y0 + (mp.nrows - 1) * step;
  const int32_t r0 = y0, r1 = std::min(last_y + step, o->height);
  const size_t off = (size_t)r0 * o->width * 3, cnt = (size_t)(r1 - r0) * o->width * 3;
  hipStream_t st = s->stream;
  HIP_TRY(hipMemcpyAsync(s->fb_scratch.p + off, fb + off, cnt * sizeof(float), hipMemcpyHostToDevice, st));
  if ((rc = render_device(s, o, mp, s->fb_scratch.p, st, nullptr, true))) return rc;
  HIP_TRY(hipMemcpyAsync(fb + off, s->fb_scratch.p + off, cnt * sizeof(float), hipMemcpyDeviceToHost, st));
  if ((rc = read_stats(s, st, &local))) return rc;
  if (out) *out = local;
  return RT_OK;
}

extern "C" int rt_render_bands_device(rt_scene* s, const rt_options* o, float* d_bands, int32_t band_h,
                                      int32_t rank, int32_t world, void* stream, rt_stats* out) {
  if (!s || !d_bands) return fail(RT_E_INVALID, "null argument");
  int rc = check_options(s, o);
  if (rc) return rc;
  if (band_h <= 0 || world <= 0 || rank < 0 || rank >= world)
    return fail(RT_E_INVALID, "bad band geometry band_h=%d rank=%d world=%d", band_h, rank, world);
  int32_t rows = 0;
  if ((rc = rt_band_rows(o->height, band_h, world, &rows))) return rc;
  Mapping mp;
  mp.mode = 1;
  mp.y0 = 0;
  mp.nrows = rows;
  mp.ncols = o->width;
  mp.step = 1;
  mp.max_step = 1;
  mp.band_h = band_h;
  mp.rank = rank;
  mp.world = world;
  std::lock_guard<std::mutex> lk(s->mu);
  DeviceGuard g(s->device);
  return render_device(s, o, mp, d_bands, (hipStream_t)stream, out);
}

extern "C" int rt_scene_last_stats(rt_scene* s, rt_stats* out) {
  if (!s || !out) return fail(RT_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(s->mu);
  if (!s->stats_kept) return fail(RT_E_INVALID, "the last render call set RT_FLAG_NO_STATS");
  DeviceGuard g(s->device);
  HIP_TRY(hipStreamWaitEvent(s->stream, s->done, 0));
  if (int rc = flush_reduce(s, s->stream)) return rc;
  return read_stats(s, s->stream, out);
}

extern "C" int rt_scene_last_timing(rt_scene* s, double* setup_ms, double* render_ms) {
  if (!s || !setup_ms || !render_ms) return fail(RT_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(s->mu);
  if (!s->timed) return fail(RT_E_INVALID, "the last render call did not set RT_FLAG_TIMING");
  DeviceGuard g(s->device);
  float a = 0.0f, b = 0.0f;
  HIP_TRY(hipEventSynchronize(s->tev[2]));
  HIP_TRY(hipEventElapsedTime(&a, s->tev[0], s->tev[1]));
  HIP_TRY(hipEventElapsedTime(&b, s->tev[1], s->tev[2]));
  *setup_ms = a;
  *render_ms = b;
  return RT_OK;
}

extern "C" int rt_unshard_bands_device(const float* d_gathered, float* d_fb, int32_t width, int32_t height,
                                       int32_t band_h, int32_t world, void* stream) {
  if (!d_gathered || !d_fb || width <= 0 || height <= 0 || band_h <= 0 || world <= 0)
    return fail(RT_E_INVALID, "bad arguments");
  const int e = rtmi_launch_unshard(d_gathered, d_fb, width, height, band_h, world, stream);
  if (e) return fail(RT_E_DEVICE, "unshard launch failed: %s", hipGetErrorString((hipError_t)e));
  return RT_OK;
}

extern "C" int64_t rt_ppm_payload_bytes(int32_t width, int32_t height, int32_t bits) {
  if (width <= 0 || height <= 0 || bits < 1 || bits > 16) return fail(RT_E_INVALID, "bad ppm size / bits");
  return (int64_t)width * height * 3 * (bits <= 8 ? 1 : 2);
}

extern "C" int rt_ppm_header(int32_t width, int32_t height, int32_t bits, char* buf, int32_t buf_len) {
  if (width <= 0 || height <= 0 || bits < 1 || bits > 16 || !buf) return fail(RT_E_INVALID, "bad arguments");
  const int n = std::snprintf(buf, (size_t)std::max(0, buf_len), "P6 %d %d %d ", width, height, (1 << bits) - 1);
  if (n < 0 || n >= buf_len) return fail(RT_E_INVALID, "header buffer too small (%d bytes)", buf_len);
  return n;
}

extern "C" int rt_ppm_encode_device(const float* d_fb, int32_t width, int32_t height, int32_t bits, int32_t srgb,
                                    void* d_out, void* stream) {
  if (!d_fb || !d_out) return fail(RT_E_INVALID, "null buffer");
  if (rt_ppm_payload_bytes(width, height, bits) < 0) return RT_E_INVALID;
  if (((uintptr_t)d_fb & 15) || ((uintptr_t)d_out & 7)) return fail(RT_E_INVALID, "buffers must be 16-B (fb) / 8-B (out) aligned");
  const int e = rtmi_launch_ppm_encode(d_fb, (long long)width * height * 3, bits, srgb ? 1 : 0, d_out, stream);
  if (e) return fail(RT_E_DEVICE, "ppm encode launch failed: %s", hipGetErrorString((hipError_t)e));
  return RT_OK;
}

extern "C" int rt_rgba_encode_device(const float* d_fb, int32_t width, int32_t height, uint8_t alpha, void* d_out,
                                     void* stream) {
  if (!d_fb || !d_out) return fail(RT_E_INVALID, "null buffer");
  if (width <= 0 || height <= 0 || width > 65536 || height > 65536)
    return fail(RT_E_INVALID, "bad image size %dx%d", width, height);
  if (((uintptr_t)d_fb & 3) || ((uintptr_t)d_out & 3)) return fail(RT_E_INVALID, "buffers must be 4-B aligned");
  const int e = rtmi_launch_rgba_encode(d_fb, (long long)width * height, alpha, d_out, stream);
  if (e) return fail(RT_E_DEVICE, "rgba encode launch failed: %s", hipGetErrorString((hipError_t)e));
  return RT_OK;
}

namespace {
// The last launch's lean / general list lengths: counted on the device by
// its k_frame_build2 (read back here, after the call completed), or the
// host's (a one-kernel launch: every group general).
int last_lists(rt_scene* s, int64_t* lean, int64_t* general) {
  if (!s->fr.counted) {
    *lean = s->last_lean;
    *general = s->last_general;
    return RT_OK;
  }
  DeviceGuard g(s->device);
  int32_t c[FC_WORDS];
  HIP_TRY(hipEventSynchronize(s->done));
  HIP_TRY(hipMemcpy(c, s->fr.ctr.p, sizeof c, hipMemcpyDeviceToHost));
  *lean = c[FC_LEAN];
  *general = c[FC_HEAVY];
  return RT_OK;
}
}  // namespace

extern "C" int rt_scene_last_split(rt_scene* s, int64_t* lean_groups, int64_t* general_groups) {
  if (!s || !lean_groups || !general_groups) return fail(RT_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(s->mu);
  return last_lists(s, lean_groups, general_groups);
}

extern "C" int rt_scene_last_lean_kernel(rt_scene* s, int32_t* kind) {
  if (!s || !kind) return fail(RT_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(s->mu);
  *kind = s->last_lean_kind;
  return RT_OK;
}

extern "C" int rt_scene_last_batch(rt_scene* s, int64_t* batched_groups, int64_t* fallback_groups) {
  if (!s || !batched_groups || !fallback_groups) return fail(RT_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(s->mu);
  *batched_groups = s->last_batched;
  if (s->last_batched < 0) {  // the general list of a two-class launch, counted on the device
    int64_t lean = 0;
    const int rc = last_lists(s, &lean, batched_groups);
    if (rc) return rc;
  }
  *fallback_groups = s->last_fallback;
  return RT_OK;
}

extern "C" int rt_scene_last_counters(rt_scene* s, rt_traversal_counters* out) {
  if (!s || !out) return fail(RT_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(s->mu);
  // a call without Stats (RT_FLAG_NO_STATS) reduced nothing: its counters
  // are not in the accumulator
  if (!s->stats_kept) return fail(RT_E_INVALID, "the last render call set RT_FLAG_NO_STATS");
  DeviceGuard g(s->device);
  unsigned long long h[kStatSlots];
  HIP_TRY(hipStreamWaitEvent(s->stream, s->done, 0));
  if (int rc = flush_reduce(s, s->stream)) return rc;
  HIP_TRY(hipStreamSynchronize(s->stream));
  HIP_TRY(hipMemcpy(h, s->acc(), sizeof h, hipMemcpyDeviceToHost));
  out->wave_node_fetches = h[STAT_NODE_FETCH];
  out->wave_tri_fetches = h[STAT_TRI_FETCH];
  out->lane_node_visits = h[STAT_LANE_NODES];
  out->lane_tri_tests = h[STAT_LANE_TRIS];
  return RT_OK;
}

// ---- test hooks (tests/test_gpu_frame.py; not part of include/rtmi.h) ----

// Pixel-list slots per pixel, 2^lg (lg >= 0: used from the next call on; the
// buffers are re-allocated): a test forces lists past their slots (the
// pixels' camera rays then take the BVH). Returns the current lg (lg < 0:
// query only).
extern "C" int rtmi_test_slot_lg(rt_scene* s, int32_t lg) {
  if (!s || lg > 10) return fail(RT_E_INVALID, "bad argument");
  std::lock_guard<std::mutex> lk(s->mu);
  if (lg >= 0) s->fr.want_lg = s->fr2.want_lg = lg;
  return s->fr.slot_lg;
}

// Whether the last render call ran its build on the scene's build stream
// (pipelined, rt_scene::pipe), and the call's buffer set (0 / 1: which of the
// two it used; it alternates between pipelined calls).
extern "C" int rtmi_test_last_pipelined(rt_scene* s, int32_t* set) {
  if (!s) return fail(RT_E_INVALID, "null scene");
  std::lock_guard<std::mutex> lk(s->mu);
  if (set) *set = s->fr.id;
  return s->pipe ? 1 : 0;
}

// The last render call's device-built camera-ray lists and pixel records
// (image-sized arrays; only the call's pixels are defined) as CSR: off:
// w*h + 1 (a pixel's true list length, overflowed ones included), ent: up to
// ent_cap entries (a pixel past its 2^lg slots contributes its first 2^lg
// entries and pads the rest with -1), info: w*h. Returns the entries
// copied, or a negative RT_E_* code.
extern "C" int64_t rtmi_test_frame_lists(rt_scene* s, int32_t* off, int32_t* ent, int64_t ent_cap, uint32_t* info) {
  if (!s || !off || !ent || !info) return fail(RT_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(s->mu);
  DeviceGuard g(s->device);
  const rt_scene::Frame& f = s->fr;
  if (!f.slots.p || f.w == 0 || f.slot_lg < 0) return fail(RT_E_INVALID, "no per-call lists yet");
  const size_t npx = (size_t)f.w * (size_t)f.h;
  HIP_TRY(hipEventSynchronize(s->done));
  HIP_TRY(hipMemcpy(info, f.info.p, npx * sizeof(uint32_t), hipMemcpyDeviceToHost));
  std::vector<int32_t> slots(npx << f.slot_lg);
  HIP_TRY(hipMemcpy(slots.data(), f.slots.p, slots.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
  const uint32_t K = 1u << f.slot_lg;
  int64_t n = 0;
  off[0] = 0;
  for (size_t p = 0; p < npx; ++p) {
    const uint32_t c = info[p] & kPixCount;
    for (uint32_t k = 0; k < c; ++k, ++n)
      if (n < ent_cap) ent[n] = k < K ? slots[(p << f.slot_lg) + k] : -1;
    off[p + 1] = (int32_t)n;
  }
  return std::min<int64_t>(n, ent_cap);
}

// Test hook: the LTri record (rt_common.h) of triangle v9 (v0, v1, v2 as 9
// doubles, mesh object space) for the shadow direction d (float64), as
// rt_scene_create builds it; out: 16 words.
extern "C" int rtmi_test_ltri(const double* v9, const double* d, int32_t face, void* out) {
  if (!v9 || !d || !out) return fail(RT_E_INVALID, "null argument");
  const double v[3][3] = {{v9[0], v9[1], v9[2]}, {v9[3], v9[4], v9[5]}, {v9[6], v9[7], v9[8]}};
  make_ltri(v, d, face, (LTri*)out);
  return RT_OK;
}

// Test hook: the last call's pixel records (w*h words, rt_frame.h: list
// length | shadow skip bits << 24; only the call's pixels are defined).
extern "C" int rtmi_test_pixel_info(rt_scene* s, uint32_t* info) {
  if (!s || !info) return fail(RT_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(s->mu);
  DeviceGuard g(s->device);
  const rt_scene::Frame& f = s->fr;
  if (!f.info.p || f.w == 0) return fail(RT_E_INVALID, "no per-call records yet");
  HIP_TRY(hipEventSynchronize(s->done));
  HIP_TRY(hipMemcpy(info, f.info.p, (size_t)f.w * (size_t)f.h * sizeof(uint32_t), hipMemcpyDeviceToHost));
  return RT_OK;
}

// The host builders (rt_bins.cpp build_pixel_bins + build_shadow_skips) on
// this scene's faces, camera and light grids: the lists and records a render
// call of this image size and bias must build on the device. off: w*h + 1,
// info: w*h. Returns the number of entries (those past ent_cap not copied),
// -1 when the host builder declines the camera.
extern "C" int64_t rtmi_test_host_lists(rt_scene* s, int32_t w, int32_t h, double bias, int32_t* off, int32_t* ent,
                                        int64_t ent_cap, uint32_t* info) {
  if (!s || !off || !ent || !info || w <= 0 || h <= 0) return fail(RT_E_INVALID, "bad argument");
  std::lock_guard<std::mutex> lk(s->mu);
  if (!s->binnable) return -1;
  PixelBinsHost hb;
  const char* why = "";
  if (!build_pixel_bins(s->bin_tris, s->mesh_o2w, s->mesh_w2o, s->c2w, s->fov, w, h, &hb, &why)) return -1;
  const size_t npx = (size_t)w * (size_t)h;
  std::vector<uint32_t> sk;
  if (!(s->skippable && build_shadow_skips(hb.off, s->skip_planes, s->mesh_w2o, s->grid_occ, s->c2w, s->fov, w, h,
                                           bias, &sk, &why)))
    sk.assign((npx + 3) / 4, 0u);
  std::copy(hb.off.begin(), hb.off.end(), off);
  const int64_t total = hb.off.back();
  std::copy(hb.ent.begin(), hb.ent.begin() + std::min<int64_t>(total, std::max<int64_t>(0, ent_cap)), ent);
  for (size_t k = 0; k < npx; ++k) {
    const uint32_t n = (uint32_t)(hb.off[k + 1] - hb.off[k]);
    info[k] = std::min<uint32_t>(n, kPixCount) | (sk[k >> 2] >> (8 * (k & 3)) & 0xffu) << 24;
  }
  return total;
}
