// rt_kernels_f64.hip — float64 (parity mode) instantiations of the render
// kernels. Built with -ffp-contract=off so every operation rounds exactly as
// the reference's (and the oracle's) IEEE float64 arithmetic does.
#include "rt_device.h"

#ifndef RTMI_PX64_P
#define RTMI_PX64_P 4  // pixels per wave batch (k_render_px64)
#endif

namespace rtmi {
template __global__ void k_render<double, false>(const RenderParams<double>);
template __global__ void k_render<double, true>(const RenderParams<double>);
template __global__ void k_render_px64<RTMI_PX64_P, 1>(const RenderParams<double>);
template __global__ void k_render_px64<RTMI_PX64_P, kMaxShadeLevels>(const RenderParams<double>);
}

namespace rtmi {
// One distant light's float64 shadow records (ShTri64) over its grid entries
// ent[0, n): the object-space shadow direction exactly as k_render_px64's
// block cache and shade_path form it (-lightDir through the mesh object's
// world_to_object, xform_xf), then tri_ref's pvec / det / invDet of it.
__global__ __launch_bounds__(256) void k_build_sh64(const DevObject<double>* objects, int mesh_obj,
                                                    const DevLight<double>* lights, int light, const int32_t* ent,
                                                    int n, const TriF64* tris, int tri_rec0, ShTri64* out) {
  using R = double;
  const int e = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (e >= n) return;
  const DevObject<R>& ob = objects[mesh_obj];
  const DevLight<R>& L = lights[light];
  const V3<R> ldir{L.v[0], L.v[1], L.v[2]};
  const V3<R> sd{ldir.x * R(-1), ldir.y * R(-1), ldir.z * R(-1)};
  const V3<R> d = xform_xf<R, false>(ob.xf, ob.w2o, sd);
  const TriF64& t = tris[(ent[e] >> 6) - tri_rec0];
  ShTri64 r;
  for (int k = 0; k < 3; ++k) {
    r.v0[k] = t.v0[k];
    r.e1[k] = t.e1[k];
    r.e2[k] = t.e2[k];
  }
  const R v0v2x = t.e2[0], v0v2y = t.e2[1], v0v2z = t.e2[2];
  r.pvec[0] = d.y * v0v2z - d.z * v0v2y;  // tri_ref (geom.nim:296-298)
  r.pvec[1] = d.z * v0v2x - d.x * v0v2z;
  r.pvec[2] = d.x * v0v2y - d.y * v0v2x;
  r.det = t.e1[0] * r.pvec[0] + t.e1[1] * r.pvec[1] + t.e1[2] * r.pvec[2];
  r.inv_det = Prec<R>::rcp(r.det);
  r.id = t.id;
  r.pad[0] = r.pad[1] = r.pad[2] = 0;
  out[e] = r;
}
}  // namespace rtmi

extern "C" int rtmi_build_sh64(const rtmi::DevObject<double>* objects, int mesh_obj, const rtmi::DevLight<double>* lights,
                               int light, const int32_t* ent, int n, const rtmi::TriF64* tris, int tri_rec0,
                               rtmi::ShTri64* out, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(rtmi::k_build_sh64, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, objects, mesh_obj,
                     lights, light, ent, n, tris, tri_rec0, out);
  return (int)hipGetLastError();
}

// px64: k_render_px64 (one pixel per wave, akGrid >= 64 spp; 1: a scene
// without reflective materials, 2: with), else k_render
extern "C" int rtmi_launch_render_f64(const rtmi::RenderParams<double>* p, int blocks, int px64, void* stream) {
  if (px64 == 1)
    hipLaunchKernelGGL((rtmi::k_render_px64<RTMI_PX64_P, 1>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, *p);
  else if (px64 == 2)
    hipLaunchKernelGGL((rtmi::k_render_px64<RTMI_PX64_P, rtmi::kMaxShadeLevels>), dim3(blocks), dim3(256), 0,
                       (hipStream_t)stream, *p);
  else if (p->flags & rtmi::RT_DEV_FLAG_COUNT)
    hipLaunchKernelGGL((rtmi::k_render<double, true>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, *p);
  else
    hipLaunchKernelGGL((rtmi::k_render<double, false>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, *p);
  return (int)hipGetLastError();
}

// resident blocks of k_render_px64 per CU (its grid: one wave per resident slot)
extern "C" int rtmi_px64_blocks_per_cu(int px64) {
  int n = 0;
  const void* k = px64 == 1 ? (const void*)rtmi::k_render_px64<RTMI_PX64_P, 1>
                            : (const void*)rtmi::k_render_px64<RTMI_PX64_P, rtmi::kMaxShadeLevels>;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 256, 0) != hipSuccess) return 0;
  return n;
}

// pixels per wave batch of k_render_px64 (the grid covers nbatch = pixels / P)
extern "C" int rtmi_px64_batch() { return RTMI_PX64_P; }
