// rt_kernels_f64.hip — float64 (parity mode) instantiation of the render
// kernel. Built with -ffp-contract=off so every operation rounds exactly as
// the reference's (and the oracle's) IEEE float64 arithmetic does.
#include "rt_device.h"

namespace rtmi {
template __global__ void k_render<double, false>(const RenderParams<double>);
template __global__ void k_render<double, true>(const RenderParams<double>);
}

extern "C" int rtmi_launch_render_f64(const rtmi::RenderParams<double>* p, int blocks, void* stream) {
  if (p->flags & rtmi::RT_DEV_FLAG_COUNT)
    hipLaunchKernelGGL((rtmi::k_render<double, true>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, *p);
  else
    hipLaunchKernelGGL((rtmi::k_render<double, false>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, *p);
  return (int)hipGetLastError();
}
