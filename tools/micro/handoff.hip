// Cross-stream hand-off latency on one GPU: kernel A (stream a) -> kernel B
// (stream b), ordered by (0) hipEventRecord / hipStreamWaitEvent, or (1)
// hipStreamWriteValue32 / hipStreamWaitValue32, or (2) the same stream.
// Each kernel records its start / end with s_memrealtime (100 MHz); prints
// the median gap from A's end to B's start in microseconds.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

__global__ void k_spin(unsigned long long* ts, int slot, long long spin) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) ts[2 * slot] = t0;
  long long x = 0;
  for (long long i = 0; i < spin; ++i) x += i ^ (long long)threadIdx.x;
  if (x == 42) ts[1023] = (unsigned long long)x;
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(&ts[2 * slot + 1], __builtin_amdgcn_s_memrealtime());
}

int main() {
  unsigned long long* ts;
  unsigned int* flag;
  unsigned int* sflag = nullptr;
  hipMalloc(&ts, 1024 * 8);
  hipMalloc(&flag, 64);
  if (hipExtMallocWithFlags((void**)&sflag, 8, hipMallocSignalMemory) != hipSuccess) printf("no signal memory\n");
  hipStream_t a, b;
  hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
  hipEvent_t ev;
  hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  for (int mode = 0; mode < 4; ++mode) {
    std::vector<double> gaps;
    for (int rep = 0; rep < 40; ++rep) {
      hipMemset(ts, 0, 1024 * 8);
      hipMemset(flag, 0, 64);
      if (sflag) hipMemset(sflag, 0, 8);
      hipDeviceSynchronize();
      hipStream_t sb = mode == 2 ? a : b;
      // B is enqueued first (its wait set up before A runs), as a pipelined render is
      if (mode == 0) {
        hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, a, ts, 0, 20000LL);
        hipEventRecord(ev, a);
        hipStreamWaitEvent(b, ev, 0);
      } else if (mode == 3) {
        hipStreamWaitValue32(b, sflag, (unsigned)(rep + 1), hipStreamWaitValueGte, 0xffffffffu);
        hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, a, ts, 0, 20000LL);
        hipStreamWriteValue32(a, sflag, (unsigned)(rep + 1), 0);
      } else if (mode == 1) {
        hipStreamWaitValue32(b, flag, (unsigned)(rep + 1), hipStreamWaitValueGte, 0xffffffffu);
        hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, a, ts, 0, 20000LL);
        hipStreamWriteValue32(a, flag, (unsigned)(rep + 1), 0);
      } else {
        hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, a, ts, 0, 20000LL);
      }
      hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, sb, ts, 1, 2000LL);
      hipDeviceSynchronize();
      unsigned long long h[4];
      hipMemcpy(h, ts, 32, hipMemcpyDeviceToHost);
      gaps.push_back(((double)h[2] - (double)h[1]) / 100.0);  // 100 MHz ticks -> us
    }
    std::sort(gaps.begin(), gaps.end());
    printf("mode %d (%s): median gap %.2f us, p10 %.2f, p90 %.2f\n", mode,
           mode == 0 ? "event" : mode == 1 ? "write/wait value" : mode == 2 ? "same stream" : "write/wait value, signal memory", gaps[gaps.size() / 2],
           gaps[gaps.size() / 10], gaps[gaps.size() * 9 / 10]);
  }
  return 0;
}
