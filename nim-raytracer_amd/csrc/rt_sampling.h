// rt_sampling.h — the stochastic antialias samplers of sampling.nim:21-113
// (jitteredGrid, multiJittered, correlatedMultiJittered, each called with
// (m, m) by renderer.nim:189-202) over a counter-based RNG.
//
// The reference draws from Nim's `random`, seeded from the clock
// (renderer.nim:215 `randomize()`), so its stochastic images are not
// reproducible. Here every draw is a pure function of (rt_options.seed,
// absolute pixel (x, y), draw index): SplitMix64 finalisers over a Weyl
// sequence. Draw k of pixel (x, y) does not depend on which lane, band or
// progressive pass renders the pixel, and the device can build a table in
// parallel. The ORDER of the draws is the reference's loop order (the oracle,
// oracle/rt_oracle.c sample_table, states it sequentially):
//   jitteredGrid          2 draws per (j, i), row-major;
//   multiJittered         2 per (j, i) canonical, then one per (j, i) for the
//                         x shuffle, then one per (i, j), i outer, for y;
//   correlatedMultiJitter same canonical, one per row j (x), one per column i (y).
// random(x) = u * x with u uniform in [0, 1) (53 bits); `.int` truncates.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD inline
#endif

namespace rtmi {

RT_HD uint64_t rng_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
RT_HD uint64_t rng_pixel_key(uint64_t seed, int32_t x, int32_t y) {
  return rng_mix64(seed ^ rng_mix64(((uint64_t)(uint32_t)y << 32) | (uint32_t)x));
}
RT_HD double rng_draw(uint64_t key, uint64_t k) {
  return (double)(rng_mix64(key + (k + 1) * 0x9E3779B97F4A7C15ULL) >> 11) * (1.0 / 9007199254740992.0);
}
// the shuffles' `k = j + (random(1.0) * (n - j).float).int`, in float64
RT_HD int32_t rng_pick(double u, int32_t j, int32_t n) { return j + (int32_t)(u * (double)(n - j)); }

// jitteredGrid entry e = j*m + i (sampling.nim:21-33): offsets in [0, 1)
RT_HD void jittered_entry(uint64_t key, int32_t m, int32_t e, double& sx, double& sy) {
  const int32_t j = e / m, i = e - j * m;
  const double xs = 1.0 / (double)m, ys = 1.0 / (double)m;
  sx = (double)i * xs + rng_draw(key, 2 * (uint64_t)e) * xs;
  sy = (double)j * ys + rng_draw(key, 2 * (uint64_t)e + 1) * ys;
}
// multiJittered / correlatedMultiJittered canonical entry (sampling.nim:46-52)
RT_HD void canonical_entry(uint64_t key, int32_t m, int32_t e, double& sx, double& sy) {
  const int32_t j = e / m, i = e - j * m;
  const double xs = 1.0 / (double)m, ys = 1.0 / (double)m;
  sx = ((double)i + ((double)j + rng_draw(key, 2 * (uint64_t)e)) * xs) * ys;
  sy = ((double)j + ((double)i + rng_draw(key, 2 * (uint64_t)e + 1)) * ys) * xs;
}

// The whole (m, m) table of a stochastic kind, sequentially (one lane), in
// p[j*m + i] order: sx[0 .. m*m), sy[0 .. m*m). T = double (parity) or float.
template <class T>
RT_HD void sample_table_seq(int32_t kind, int32_t m, uint64_t key, T* sx, T* sy) {
  const int32_t n = m, len = m * m;
  for (int32_t e = 0; e < len; ++e) {
    double a, b;
    if (kind == 2) jittered_entry(key, m, e, a, b);
    else canonical_entry(key, m, e, a, b);
    sx[e] = (T)a;
    sy[e] = (T)b;
  }
  if (kind == 2) return;
  const uint64_t bx = 2 * (uint64_t)len;
  if (kind == 3) {  // multiJittered (sampling.nim:55-74)
    const uint64_t by = bx + (uint64_t)len;
    for (int32_t j = 0; j < n; ++j)
      for (int32_t i = 0; i < m; ++i) {
        const int32_t k = rng_pick(rng_draw(key, bx + (uint64_t)j * m + i), j, n);
        const T t = sx[j * m + i];
        sx[j * m + i] = sx[k * m + i];
        sx[k * m + i] = t;
      }
    for (int32_t i = 0; i < m; ++i)
      for (int32_t j = 0; j < n; ++j) {
        const int32_t k = rng_pick(rng_draw(key, by + (uint64_t)i * n + j), i, m);
        const T t = sy[j * m + i];
        sy[j * m + i] = sy[j * m + k];
        sy[j * m + k] = t;
      }
  } else {  // correlatedMultiJittered (sampling.nim:92-111)
    const uint64_t by = bx + (uint64_t)n;
    for (int32_t j = 0; j < n; ++j) {
      const int32_t k = rng_pick(rng_draw(key, bx + (uint64_t)j), j, n);
      for (int32_t i = 0; i < m; ++i) {
        const T t = sx[j * m + i];
        sx[j * m + i] = sx[k * m + i];
        sx[k * m + i] = t;
      }
    }
    for (int32_t i = 0; i < m; ++i) {
      const int32_t k = rng_pick(rng_draw(key, by + (uint64_t)i), i, m);
      for (int32_t j = 0; j < n; ++j) {
        const T t = sy[j * m + i];
        sy[j * m + i] = sy[j * m + k];
        sy[j * m + k] = t;
      }
    }
  }
}

}  // namespace rtmi
