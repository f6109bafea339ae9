// rt_multi.cpp — one process, several GPUs: rt_render_frame_multi (SURVEY.md
// 8(b) "8-GPU shard plus gather"), for callers without a process per GPU
// (the Nim renderer is one process; the bench's torch.distributed path in
// rtmi/dist.py is the one-process-per-GPU form of the same layout).
//
//  * the scene is replicated: one rt_scene per entry of the device list
//    (built once, concurrently usable);
//  * image rows are cut into band_h-row bands dealt round-robin, band b to
//    rank b % world (rt_render_bands_device), every rank rendering on its
//    own device and stream at the same time;
//  * the compact band buffers move to the first device over xGMI
//    (hipMemcpyPeerAsync, peer access enabled where the topology allows),
//    each copy ordered after its rank's render by an event, and one
//    rt_unshard_bands_device launch assembles the frame there;
//  * Stats are summed over ranks (rt_scene_last_stats).
// A device may be listed more than once (several ranks on one GPU): the
// layout, copies and un-interleave are then exercised on a one-GPU machine
// (tests/test_gpu_multi.py).
#include <hip/hip_runtime.h>

#include <mutex>
#include <string>
#include <vector>

#include "../../include/rtmi.h"
#include "rt_common.h"

struct rt_multi {
  std::mutex mu;
  int32_t band_h = 4;
  std::vector<int> dev;
  std::vector<rt_scene*> scene;
  std::vector<hipStream_t> stream;
  std::vector<hipEvent_t> done;
  std::vector<float*> bands;  // per rank, on its device
  size_t band_floats = 0;
  float* gathered = nullptr;  // world * band_floats on dev[0]
  float* frame = nullptr;     // w * h * 3 on dev[0] (host-framebuffer form)
  size_t frame_floats = 0;

  void release() {
    for (size_t i = 0; i < dev.size(); ++i) {
      (void)hipSetDevice(dev[i]);
      if (i < stream.size() && stream[i]) (void)hipStreamSynchronize(stream[i]);
      if (i < bands.size() && bands[i]) (void)hipFree(bands[i]);
      if (i < done.size() && done[i]) (void)hipEventDestroy(done[i]);
      if (i < stream.size() && stream[i]) (void)hipStreamDestroy(stream[i]);
      if (i < scene.size() && scene[i]) (void)rt_scene_destroy(scene[i]);
    }
    if (!dev.empty()) {
      (void)hipSetDevice(dev[0]);
      if (gathered) (void)hipFree(gathered);
      if (frame) (void)hipFree(frame);
    }
    bands.clear();
    gathered = frame = nullptr;
  }
};

namespace {

struct CurrentDevice {  // restores the caller's device
  int prev = -1;
  CurrentDevice() { (void)hipGetDevice(&prev); }
  ~CurrentDevice() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

#define MULTI_TRY(expr)                                                                                 \
  do {                                                                                                  \
    hipError_t e_ = (expr);                                                                             \
    if (e_ != hipSuccess) return rtmi_fail_msg(RT_E_DEVICE, (std::string(#expr ": ") + hipGetErrorString(e_)).c_str()); \
  } while (0)

int ensure_buffers(rt_multi* m, size_t band_floats, size_t frame_floats) {
  const size_t world = m->dev.size();
  if (band_floats > m->band_floats) {
    for (size_t i = 0; i < world; ++i) {
      MULTI_TRY(hipSetDevice(m->dev[i]));
      MULTI_TRY(hipStreamSynchronize(m->stream[i]));
      if (m->bands[i]) MULTI_TRY(hipFree(m->bands[i]));
      m->bands[i] = nullptr;
      MULTI_TRY(hipMalloc((void**)&m->bands[i], band_floats * sizeof(float)));
    }
    MULTI_TRY(hipSetDevice(m->dev[0]));
    if (m->gathered) MULTI_TRY(hipFree(m->gathered));
    m->gathered = nullptr;
    MULTI_TRY(hipMalloc((void**)&m->gathered, world * band_floats * sizeof(float)));
    m->band_floats = band_floats;
  }
  if (frame_floats > m->frame_floats) {
    MULTI_TRY(hipSetDevice(m->dev[0]));
    MULTI_TRY(hipStreamSynchronize(m->stream[0]));
    if (m->frame) MULTI_TRY(hipFree(m->frame));
    m->frame = nullptr;
    MULTI_TRY(hipMalloc((void**)&m->frame, frame_floats * sizeof(float)));
    m->frame_floats = frame_floats;
  }
  return RT_OK;
}

// Renders every rank's bands, gathers them on dev[0] and un-interleaves into
// d_fb (on dev[0]); the result is complete on stream[0].
int frame_device(rt_multi* m, const rt_options* o, float* d_fb, rt_stats* out) {
  const int world = (int)m->dev.size();
  int32_t rows = 0;
  int rc = rt_band_rows(o->height, m->band_h, world, &rows);
  if (rc) return rc;
  const size_t n = (size_t)rows * o->width * 3;
  if ((rc = ensure_buffers(m, n, 0))) return rc;
  for (int i = 0; i < world; ++i) {  // all ranks in flight at once
    MULTI_TRY(hipSetDevice(m->dev[i]));
    if ((rc = rt_render_bands_device(m->scene[i], o, m->bands[i], m->band_h, i, world, m->stream[i], nullptr)))
      return rc;
    MULTI_TRY(hipEventRecord(m->done[i], m->stream[i]));
  }
  MULTI_TRY(hipSetDevice(m->dev[0]));
  for (int i = 0; i < world; ++i) {
    MULTI_TRY(hipStreamWaitEvent(m->stream[0], m->done[i], 0));
    float* dst = m->gathered + (size_t)i * n;
    if (m->dev[i] == m->dev[0])
      MULTI_TRY(hipMemcpyAsync(dst, m->bands[i], n * sizeof(float), hipMemcpyDeviceToDevice, m->stream[0]));
    else
      MULTI_TRY(hipMemcpyPeerAsync(dst, m->dev[0], m->bands[i], m->dev[i], n * sizeof(float), m->stream[0]));
  }
  if ((rc = rt_unshard_bands_device(m->gathered, d_fb, o->width, o->height, m->band_h, world, m->stream[0])))
    return rc;
  if (out) {
    rt_stats tot{};
    for (int i = 0; i < world; ++i) {
      rt_stats st{};
      if ((rc = rt_scene_last_stats(m->scene[i], &st))) return rc;
      tot.num_primary_rays += st.num_primary_rays;
      tot.num_intersection_tests += st.num_intersection_tests;
      tot.num_intersection_hits += st.num_intersection_hits;
      tot.num_shadow_rays += st.num_shadow_rays;
      tot.num_reflection_rays += st.num_reflection_rays;
    }
    *out = tot;
  }
  return RT_OK;
}

}  // namespace

extern "C" {

int rt_multi_create(const rt_scene_desc* desc, const int32_t* devices, int32_t num_devices, int32_t band_h,
                    rt_multi** out) {
  if (!desc || !out || (num_devices > 0 && !devices)) return rtmi_fail_msg(RT_E_INVALID, "null argument");
  *out = nullptr;
  if (num_devices <= 0 || num_devices > 64) return rtmi_fail_msg(RT_E_INVALID, "num_devices must be 1..64");
  if (band_h < 0) return rtmi_fail_msg(RT_E_INVALID, "negative band_h");
  const int have = rt_device_count();
  if (have <= 0) return rtmi_fail_msg(RT_E_DEVICE, "no HIP device");
  for (int i = 0; i < num_devices; ++i)
    if (devices[i] < 0 || devices[i] >= have) return rtmi_fail_msg(RT_E_INVALID, "device index out of range");
  CurrentDevice keep;
  rt_multi* m = new rt_multi();
  m->band_h = band_h ? band_h : 4;
  m->dev.assign(devices, devices + num_devices);
  m->scene.assign((size_t)num_devices, nullptr);
  m->stream.assign((size_t)num_devices, nullptr);
  m->done.assign((size_t)num_devices, nullptr);
  m->bands.assign((size_t)num_devices, nullptr);
  int rc = RT_OK;
  for (int i = 0; i < num_devices && rc == RT_OK; ++i) {
    if (hipSetDevice(m->dev[(size_t)i]) != hipSuccess ||
        hipStreamCreateWithFlags(&m->stream[(size_t)i], hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&m->done[(size_t)i], hipEventDisableTiming) != hipSuccess) {
      rc = rtmi_fail_msg(RT_E_DEVICE, "stream / event creation failed");
      break;
    }
    rc = rt_scene_create(desc, &m->scene[(size_t)i]);
  }
  // direct xGMI copies from every other device into the first
  for (int i = 1; i < num_devices && rc == RT_OK; ++i) {
    const int a = m->dev[0], b = m->dev[(size_t)i];
    int can = 0;
    if (a != b && hipDeviceCanAccessPeer(&can, a, b) == hipSuccess && can) {
      (void)hipSetDevice(a);
      const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) rc = rtmi_fail_msg(RT_E_DEVICE, "peer access");
      (void)hipGetLastError();
    }
  }
  if (rc != RT_OK) {
    m->release();
    delete m;
    return rc;
  }
  *out = m;
  return RT_OK;
}

int rt_render_frame_multi_device(rt_multi* m, const rt_options* opts, float* d_fb, rt_stats* out) {
  if (!m || !opts || !d_fb) return rtmi_fail_msg(RT_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(m->mu);
  CurrentDevice keep;
  int rc = frame_device(m, opts, d_fb, out);
  if (rc) return rc;
  if (out) MULTI_TRY(hipStreamSynchronize(m->stream[0]));
  return RT_OK;
}

int rt_render_frame_multi(rt_multi* m, const rt_options* opts, float* fb, int32_t fb_w, int32_t fb_h,
                          rt_stats* out) {
  if (!m || !opts || !fb) return rtmi_fail_msg(RT_E_INVALID, "null argument");
  if (fb_w != opts->width || fb_h != opts->height)
    return rtmi_fail_msg(RT_E_INVALID, "framebuffer size does not match the options");
  std::lock_guard<std::mutex> lk(m->mu);
  CurrentDevice keep;
  const size_t nf = (size_t)opts->width * opts->height * 3;
  int rc = ensure_buffers(m, 0, nf);
  if (rc) return rc;
  if ((rc = frame_device(m, opts, m->frame, out))) return rc;
  MULTI_TRY(hipSetDevice(m->dev[0]));
  MULTI_TRY(hipMemcpyAsync(fb, m->frame, nf * sizeof(float), hipMemcpyDeviceToHost, m->stream[0]));
  MULTI_TRY(hipStreamSynchronize(m->stream[0]));
  return RT_OK;
}

int rt_multi_set_camera(rt_multi* m, const double camera_to_world[16], double fov_deg) {
  if (!m) return rtmi_fail_msg(RT_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(m->mu);
  CurrentDevice keep;
  for (rt_scene* s : m->scene) {
    const int rc = rt_scene_set_camera(s, camera_to_world, fov_deg);
    if (rc) return rc;
  }
  return RT_OK;
}

int rt_multi_destroy(rt_multi* m) {
  if (!m) return rtmi_fail_msg(RT_E_INVALID, "null argument");
  {
    CurrentDevice keep;
    m->release();
  }
  delete m;
  return RT_OK;
}

}  // extern "C"
