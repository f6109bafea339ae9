// rt_kernels_f32_part.hip — the float32 render kernel specialised for scene
// feature subsets (rt_fast.h F_* bits). Compiled 16 times (Makefile,
// -DRTMI_PART=0..15), each object instantiating 8 of the 128 subsets of
// {sphere, box, mesh, general transform, point light, reflection,
// stochastic sampling}; the plane is always included. The host launches the exact subset a scene uses
// (rtmi.cpp scene_features), so e.g. the mesh + plane scenes of C3-C5 run
// without the sphere / box / rotation / point-light / reflection code paths
// (fewer branches, fewer SALU, 66 instead of 72+ VGPRs).
#include "rt_fast.h"

#ifndef RTMI_PART
#error "compile with -DRTMI_PART=<0..15>"
#endif

namespace {

using rtmi::FastParams;
namespace f = rtmi::fast;

constexpr unsigned subset_mask(unsigned i) {
  return f::F_PLANE | ((i & 1u) ? f::F_SPHERE : 0u) | ((i & 2u) ? f::F_BOX : 0u) | ((i & 4u) ? f::F_MESH : 0u) |
         ((i & 8u) ? f::F_XF_GENERAL : 0u) | ((i & 16u) ? f::F_POINT : 0u) | ((i & 32u) ? f::F_REFLECT : 0u) |
         ((i & 64u) ? f::F_STOCHASTIC : 0u);
}

template <unsigned I>
int launch_one(const FastParams* p, int blocks, size_t shmem, void* stream) {
  hipLaunchKernelGGL((f::k_render_fast<false, subset_mask(I)>), dim3(blocks), dim3(256), shmem, (hipStream_t)stream,
                     *p);
  return (int)hipGetLastError();
}

template <unsigned I>
int occupancy_one(size_t shmem) {
  int nb = 0;
  const hipError_t e =
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f::k_render_fast<false, subset_mask(I)>, 256, shmem);
  return e == hipSuccess && nb > 0 ? nb : 1;
}

// the lean-pixel kernel exists for the subsets whose scenes can have lean
// pixels: a mesh, no reflection, no point light (rtmi.cpp split_lists)
constexpr bool has_lean(unsigned i) { return (i & 4u) && !(i & 32u) && !(i & 16u); }

template <unsigned I>
int launch_lean_one(const FastParams* p, int blocks, size_t shmem, void* stream) {
  if constexpr (has_lean(I)) {
    hipLaunchKernelGGL((f::k_render_lean<subset_mask(I)>), dim3(blocks), dim3(256), shmem, (hipStream_t)stream, *p);
    return (int)hipGetLastError();
  } else {
    return (int)hipErrorInvalidDeviceFunction;
  }
}

template <unsigned I>
int occupancy_lean_one(size_t shmem) {
  if constexpr (has_lean(I)) {
    int nb = 0;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f::k_render_lean<subset_mask(I)>, 256, shmem);
    return e == hipSuccess && nb > 0 ? nb : 1;
  } else {
    return 0;
  }
}

template <unsigned I>
int launch_gen_one(const FastParams* p, int blocks, size_t shmem, void* stream) {
  if constexpr (has_lean(I)) {
    hipLaunchKernelGGL((f::k_render_gen<subset_mask(I)>), dim3(blocks), dim3(256), shmem, (hipStream_t)stream, *p);
    return (int)hipGetLastError();
  } else {
    return (int)hipErrorInvalidDeviceFunction;
  }
}

template <unsigned I>
int occupancy_gen_one(size_t shmem) {
  if constexpr (has_lean(I)) {
    int nb = 0;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f::k_render_gen<subset_mask(I)>, 256, shmem);
    return e == hipSuccess && nb > 0 ? nb : 1;
  } else {
    return 0;
  }
}

// the reflection-compacting kernel exists for the reflective subsets
constexpr bool has_wave(unsigned i) { return (i & 32u) != 0u; }

template <unsigned I>
int launch_wave_one(const FastParams* p, int blocks, size_t shmem, void* stream) {
  if constexpr (has_wave(I)) {
    hipLaunchKernelGGL((f::k_render_wave<subset_mask(I)>), dim3(blocks), dim3(256), shmem, (hipStream_t)stream, *p);
    return (int)hipGetLastError();
  } else {
    return (int)hipErrorInvalidDeviceFunction;
  }
}

template <unsigned I>
int occupancy_wave_one(size_t shmem) {
  if constexpr (has_wave(I)) {
    int nb = 0;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f::k_render_wave<subset_mask(I)>, 256, shmem);
    return e == hipSuccess && nb > 0 ? nb : 1;
  } else {
    return 0;
  }
}

constexpr unsigned B = RTMI_PART * 8u;

}  // namespace

#define RTMI_CAT2(a, b) a##b
#define RTMI_CAT(a, b) RTMI_CAT2(a, b)

// subset index i (0..127) -> launch; i >> 3 selects the part
extern "C" int RTMI_CAT(rtmi_launch_render_f32_part, RTMI_PART)(unsigned i, const FastParams* p, int blocks,
                                                                 size_t shmem, void* stream) {
  switch (i & 7u) {
    case 0: return launch_one<B + 0>(p, blocks, shmem, stream);
    case 1: return launch_one<B + 1>(p, blocks, shmem, stream);
    case 2: return launch_one<B + 2>(p, blocks, shmem, stream);
    case 3: return launch_one<B + 3>(p, blocks, shmem, stream);
    case 4: return launch_one<B + 4>(p, blocks, shmem, stream);
    case 5: return launch_one<B + 5>(p, blocks, shmem, stream);
    case 6: return launch_one<B + 6>(p, blocks, shmem, stream);
    default: return launch_one<B + 7>(p, blocks, shmem, stream);
  }
}

extern "C" int RTMI_CAT(rtmi_render_f32_part_blocks_per_cu, RTMI_PART)(unsigned i, size_t shmem) {
  switch (i & 7u) {
    case 0: return occupancy_one<B + 0>(shmem);
    case 1: return occupancy_one<B + 1>(shmem);
    case 2: return occupancy_one<B + 2>(shmem);
    case 3: return occupancy_one<B + 3>(shmem);
    case 4: return occupancy_one<B + 4>(shmem);
    case 5: return occupancy_one<B + 5>(shmem);
    case 6: return occupancy_one<B + 6>(shmem);
    default: return occupancy_one<B + 7>(shmem);
  }
}

extern "C" int RTMI_CAT(rtmi_launch_lean_f32_part, RTMI_PART)(unsigned i, const FastParams* p, int blocks, size_t shmem,
                                                              void* stream) {
  switch (i & 7u) {
    case 0: return launch_lean_one<B + 0>(p, blocks, shmem, stream);
    case 1: return launch_lean_one<B + 1>(p, blocks, shmem, stream);
    case 2: return launch_lean_one<B + 2>(p, blocks, shmem, stream);
    case 3: return launch_lean_one<B + 3>(p, blocks, shmem, stream);
    case 4: return launch_lean_one<B + 4>(p, blocks, shmem, stream);
    case 5: return launch_lean_one<B + 5>(p, blocks, shmem, stream);
    case 6: return launch_lean_one<B + 6>(p, blocks, shmem, stream);
    default: return launch_lean_one<B + 7>(p, blocks, shmem, stream);
  }
}

extern "C" int RTMI_CAT(rtmi_lean_f32_part_blocks_per_cu, RTMI_PART)(unsigned i, size_t shmem) {
  switch (i & 7u) {
    case 0: return occupancy_lean_one<B + 0>(shmem);
    case 1: return occupancy_lean_one<B + 1>(shmem);
    case 2: return occupancy_lean_one<B + 2>(shmem);
    case 3: return occupancy_lean_one<B + 3>(shmem);
    case 4: return occupancy_lean_one<B + 4>(shmem);
    case 5: return occupancy_lean_one<B + 5>(shmem);
    case 6: return occupancy_lean_one<B + 6>(shmem);
    default: return occupancy_lean_one<B + 7>(shmem);
  }
}

// the batched general-pixel kernel (same subsets as the lean kernel)
extern "C" int RTMI_CAT(rtmi_launch_gen_f32_part, RTMI_PART)(unsigned i, const FastParams* p, int blocks, size_t shmem,
                                                             void* stream) {
  switch (i & 7u) {
    case 0: return launch_gen_one<B + 0>(p, blocks, shmem, stream);
    case 1: return launch_gen_one<B + 1>(p, blocks, shmem, stream);
    case 2: return launch_gen_one<B + 2>(p, blocks, shmem, stream);
    case 3: return launch_gen_one<B + 3>(p, blocks, shmem, stream);
    case 4: return launch_gen_one<B + 4>(p, blocks, shmem, stream);
    case 5: return launch_gen_one<B + 5>(p, blocks, shmem, stream);
    case 6: return launch_gen_one<B + 6>(p, blocks, shmem, stream);
    default: return launch_gen_one<B + 7>(p, blocks, shmem, stream);
  }
}

extern "C" int RTMI_CAT(rtmi_gen_f32_part_blocks_per_cu, RTMI_PART)(unsigned i, size_t shmem) {
  switch (i & 7u) {
    case 0: return occupancy_gen_one<B + 0>(shmem);
    case 1: return occupancy_gen_one<B + 1>(shmem);
    case 2: return occupancy_gen_one<B + 2>(shmem);
    case 3: return occupancy_gen_one<B + 3>(shmem);
    case 4: return occupancy_gen_one<B + 4>(shmem);
    case 5: return occupancy_gen_one<B + 5>(shmem);
    case 6: return occupancy_gen_one<B + 6>(shmem);
    default: return occupancy_gen_one<B + 7>(shmem);
  }
}

// the reflection-compacting kernel (same subsets as k_render_fast's reflective ones)
extern "C" int RTMI_CAT(rtmi_launch_wave_f32_part, RTMI_PART)(unsigned i, const FastParams* p, int blocks, size_t shmem,
                                                              void* stream) {
  switch (i & 7u) {
    case 0: return launch_wave_one<B + 0>(p, blocks, shmem, stream);
    case 1: return launch_wave_one<B + 1>(p, blocks, shmem, stream);
    case 2: return launch_wave_one<B + 2>(p, blocks, shmem, stream);
    case 3: return launch_wave_one<B + 3>(p, blocks, shmem, stream);
    case 4: return launch_wave_one<B + 4>(p, blocks, shmem, stream);
    case 5: return launch_wave_one<B + 5>(p, blocks, shmem, stream);
    case 6: return launch_wave_one<B + 6>(p, blocks, shmem, stream);
    default: return launch_wave_one<B + 7>(p, blocks, shmem, stream);
  }
}

extern "C" int RTMI_CAT(rtmi_wave_f32_part_blocks_per_cu, RTMI_PART)(unsigned i, size_t shmem) {
  switch (i & 7u) {
    case 0: return occupancy_wave_one<B + 0>(shmem);
    case 1: return occupancy_wave_one<B + 1>(shmem);
    case 2: return occupancy_wave_one<B + 2>(shmem);
    case 3: return occupancy_wave_one<B + 3>(shmem);
    case 4: return occupancy_wave_one<B + 4>(shmem);
    case 5: return occupancy_wave_one<B + 5>(shmem);
    case 6: return occupancy_wave_one<B + 6>(shmem);
    default: return occupancy_wave_one<B + 7>(shmem);
  }
}
