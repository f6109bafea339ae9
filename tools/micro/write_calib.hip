// WRITE_SIZE calibration for the framebuffer's store pattern (MI355X guide:
// WRITE_SIZE is exact only for 16-B-per-lane streaming stores; other widths
// uncalibrated). Each kernel writes the same 1920 x 1080 x 3 float32 frame
// (24,883,200 B) once:
//   k_store16  — 16 B per lane (float4), the calibrated pattern;
//   k_store12  — 12 B per lane (one pixel's RGB as three dwords, consecutive
//                lanes consecutive pixels), the render kernels' finish_item;
//   k_store12q — 12 B per lane in 2 x 2 pixel tiles (a wave's 16 pixels as
//                four 2 x 2 tiles side by side: two 24-B row pieces per tile),
//                C2's k_render_fast placement.
//   rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_store -- ./write_calib
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int W = 1920, H = 1080;

__global__ void k_store16(float4* out, int n4) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n4) out[i] = make_float4(1.0f, 2.0f, 3.0f, (float)i);
}

__global__ void k_store12(float* out, int npx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < npx) {
    out[3 * (size_t)i] = 1.0f;
    out[3 * (size_t)i + 1] = 2.0f;
    out[3 * (size_t)i + 2] = (float)i;
  }
}

// pixel of thread i: tile t = i / 4 (2 x 2 tiles in row-major tile order),
// q = i % 4 its quadrant
__global__ void k_store12q(float* out, int npx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < npx) {
    const int t = i >> 2, q = i & 3;
    const int tx = t % (W / 2), ty = t / (W / 2);
    const int x = 2 * tx + (q & 1), y = 2 * ty + (q >> 1);
    const size_t p = (size_t)y * W + x;
    out[3 * p] = 1.0f;
    out[3 * p + 1] = 2.0f;
    out[3 * p + 2] = (float)i;
  }
}

int main() {
  const int npx = W * H;
  float* d = nullptr;
  if (hipMalloc(&d, (size_t)npx * 12) != hipSuccess) return 1;
  for (int rep = 0; rep < 3; ++rep) {
    k_store16<<<(npx * 3 / 4 + 255) / 256, 256>>>((float4*)d, npx * 3 / 4);
    k_store12<<<(npx + 255) / 256, 256>>>(d, npx);
    k_store12q<<<(npx + 255) / 256, 256>>>(d, npx);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::printf("frame bytes %d\n", npx * 12);
  (void)hipFree(d);
  return 0;
}
