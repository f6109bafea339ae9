// Issue-rate microbenchmark: SALU vs VALU vs mixed streams at 8 waves/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#define S4(r) "s_mul_i32 " r ", " r ", 3\n"
#define V4(r) "v_add_u32 " r ", 1, " r "\n"
template <int MODE>
__global__ __launch_bounds__(256) void k(int iters, int* out) {
  int a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
  int sa = blockIdx.x, sb = sa + 1, sc = sa + 2, sd = sa + 3;
  for (int i = 0; i < iters; ++i) {
    if (MODE == 0)  // 32 SALU
      asm volatile(
#define SB S4("%0") S4("%1") S4("%2") S4("%3")
          SB SB SB SB SB SB SB SB : "+s"(sa), "+s"(sb), "+s"(sc), "+s"(sd));
    if (MODE == 1)  // 32 VALU
      asm volatile(
#define VB V4("%0") V4("%1") V4("%2") V4("%3")
          VB VB VB VB VB VB VB VB : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    if (MODE == 2) {  // 32 SALU + 32 VALU interleaved
#define VB2 V4("%4") V4("%5") V4("%6") V4("%7")
      asm volatile(SB VB2 SB VB2 SB VB2 SB VB2 SB VB2 SB VB2 SB VB2 SB VB2
                   : "+s"(sa), "+s"(sb), "+s"(sc), "+s"(sd), "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    }
  }
  if (a + b + c + d + sa + sb + sc + sd == 12345) out[0] = 1;
}
int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  int* out; hipMalloc(&out, 4);
  hipDeviceProp_t pr; hipGetDeviceProperties(&pr, 0);
  const int cus = pr.multiProcessorCount, iters = 20000;
  for (int wps = 1; wps <= 8; wps *= 2) {
    const int blocks = cus * wps;  // 4 waves per block -> wps waves per SIMD
    for (int mode = 0; mode < 3; ++mode) {
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      auto launch = [&] {
        if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, iters, out);
        if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, iters, out);
        if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, iters, out);
      };
      launch(); hipDeviceSynchronize();
      hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double clk = 2.4e9;  // nominal
      const double insts_per_wave = (double)iters * (mode == 2 ? 64 : 32);
      const double cyc = ms * 1e-3 * clk;
      printf("waves/SIMD %d mode %s: %.3f ms, %.2f cycles per instruction per SIMD (all waves), %.2f per CU\n", wps,
             mode == 0 ? "SALU " : mode == 1 ? "VALU " : "mixed", ms, cyc / (insts_per_wave * wps), cyc / (insts_per_wave * wps * 4));
    }
  }
  return 0;
}
