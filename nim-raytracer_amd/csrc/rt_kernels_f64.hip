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
