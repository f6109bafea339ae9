// rt_kernels_io.hip — output post-pass: writePpm's per-component quantisation
// (src/utils/framebuf.nim:55-93, linearToSRGB src/utils/color.nim:17-22) on
// the GPU, so a 4K frame leaves the device as 25 / 50 MB of PPM payload
// instead of 100 MB of float32. Compiled with -ffp-contract=off: the sRGB
// expression must round exactly like the oracle (oracle_ppm_outvalue).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rtmi {

// outvalue(v): clamp to [0, 1] in float32 (NaN -> 0), optional sRGB in
// float64 returning float32, then round(c * maxval) as a float32 product
// rounded half away from zero.
__device__ __forceinline__ unsigned int ppm_outvalue(float v, float maxval, bool srgb) {
  float c = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
  if (c != c) c = 0.0f;
  if (srgb) {
    const double a = 0.055, cd = (double)c;
    c = (float)(cd <= 0.0031308 ? 12.92 * cd : (1 + a) * pow(cd, 1 / 2.4) - a);
  }
  return (unsigned int)roundf(c * maxval);
}

// 8-bit: one byte per component; 16-bit: big-endian pairs (framebuf.nim:66-70).
// Four components per thread: one float4 load, one 4- or 8-byte store.
__global__ __launch_bounds__(256) void k_ppm_encode(const float* __restrict__ fb, long long n, int bits, int srgb,
                                                    unsigned char* __restrict__ out) {
  const float maxval = (float)((1 << bits) - 1);
  const long long n4 = n / 4;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(fb)[i];
    const unsigned int q0 = ppm_outvalue(v.x, maxval, srgb), q1 = ppm_outvalue(v.y, maxval, srgb),
                       q2 = ppm_outvalue(v.z, maxval, srgb), q3 = ppm_outvalue(v.w, maxval, srgb);
    if (bits <= 8) {
      reinterpret_cast<unsigned int*>(out)[i] = q0 | (q1 << 8) | (q2 << 16) | (q3 << 24);
    } else {
      const auto be = [](unsigned int q) { return ((q >> 8) & 0xffu) | ((q & 0xffu) << 8); };
      reinterpret_cast<uint2*>(out)[i] = make_uint2(be(q0) | (be(q1) << 16), be(q2) | (be(q3) << 16));
    }
  }
  for (long long i = n4 * 4 + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const unsigned int q = ppm_outvalue(fb[i], maxval, srgb);
    if (bits <= 8) {
      out[i] = (unsigned char)q;
    } else {
      out[2 * i] = (unsigned char)(q >> 8);
      out[2 * i + 1] = (unsigned char)q;
    }
  }
}

// ImageRGBA.copyFrom (src/utils/image.nim:45-54): round(c * 0xff).uint8 per
// component, no clamp (oracle_rgba_component: out-of-range keeps the low 8
// bits of the x86 int32 conversion, NaN -> INT32_MIN), alpha constant. One
// pixel per thread: three float loads, one 4-byte store.
__device__ __forceinline__ unsigned int rgba_component(float v) {
  const float r = roundf(v * 255.0f);
  const int i = (r >= -2147483648.0f && r < 2147483648.0f) ? (int)r : (int)0x80000000u;
  return (unsigned int)i & 0xffu;
}

__global__ __launch_bounds__(256) void k_rgba_encode(const float* __restrict__ fb, long long npix, unsigned int alpha,
                                                     unsigned int* __restrict__ out) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < npix; i += stride) {
    const float* c = fb + 3 * i;
    out[i] = rgba_component(c[0]) | (rgba_component(c[1]) << 8) | (rgba_component(c[2]) << 16) | (alpha << 24);
  }
}

}  // namespace rtmi

extern "C" int rtmi_launch_rgba_encode(const float* fb, long long npix, unsigned int alpha, void* out, void* stream) {
  const int blocks = (int)(npix < 256LL * 2048 ? (npix + 255) / 256 : 2048);
  hipLaunchKernelGGL(rtmi::k_rgba_encode, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, (hipStream_t)stream, fb, npix,
                     alpha & 0xffu, (unsigned int*)out);
  return (int)hipGetLastError();
}

extern "C" int rtmi_launch_ppm_encode(const float* fb, long long n, int bits, int srgb, void* out, void* stream) {
  const long long n4 = (n + 3) / 4;
  const int blocks = (int)(n4 < 256LL * 2048 ? (n4 + 255) / 256 : 2048);
  hipLaunchKernelGGL(rtmi::k_ppm_encode, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, (hipStream_t)stream, fb, n,
                     bits, srgb, (unsigned char*)out);
  return (int)hipGetLastError();
}
