/*
 * rtmi.h — C-ABI of the MI355X-native (gfx950) trace/shade backend for
 * johnnovak/nim-raytracer.
 *
 * The reference has no FFI: its hot path is the Nim proc
 *     proc renderLine*(scene: Scene, opts: Options, fb: var Framebuf,
 *                      y: Natural, step: Natural = 1, maxStep: Natural = 1): Stats
 * (src/renderer/renderer.nim:162-211) plus proc initRenderer*()
 * (src/renderer/renderer.nim:214-215), called per scanline from worker
 * threads (src/raytracer.nim:25-32, src/concurrency/workerpool.nim:99).
 * This header is what a Nim `{.importc, dynlib: "librtmi.so".}` module binds
 * in its place. Plain C types only: pointers, sizes,
 * fixed-width integers and doubles. No torch/HIP types in any signature;
 * device streams are passed as opaque `void*` (a hipStream_t; NULL is HIP's
 * null stream, exactly as in the HIP API).
 *
 * Conventions
 *  - Every entry point returns int: RT_OK (0) or a negative RT_E_* code.
 *    The message of the last failure on the calling thread is available via
 *    rt_last_error(). No entry point aborts the caller's process.
 *  - Matrices are 4x4 column-major doubles exactly as glm stores Mat4x4
 *    (m[col*4 + row]); a point transforms as m * (x, y, z, 1).
 *  - The framebuffer is the reference's Framebuf layout
 *    (src/utils/framebuf.nim:7-28): w*h*3 float32, interleaved RGB,
 *    row-major, y = 0 is the top row. Caller-owned; the library never
 *    retains caller pointers after a call returns.
 */
#ifndef RTMI_H
#define RTMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTMI_ABI_VERSION 1

/* ---- error codes ------------------------------------------------------ */
enum {
  RT_OK = 0,
  RT_E_INVALID = -1,     /* bad argument (null pointer, size, index range) */
  RT_E_UNSUPPORTED = -2, /* valid request this build does not implement    */
  RT_E_DEVICE = -3,      /* HIP runtime / kernel failure, no usable GPU    */
  RT_E_NOMEM = -4,       /* host or device allocation failed               */
  RT_E_IO = -5           /* file could not be read / parsed                */
};

/* ---- scene description (flattened once from the Nim object graph) ----- */

/* Geometry kinds: Sphere / Plane / Box / TriangleMesh (src/renderer/geom.nim:137-155). */
enum rt_geom_type { RT_SPHERE = 0, RT_PLANE = 1, RT_BOX = 2, RT_MESH = 3 };

/* Light kinds: DistantLight / PointLight (src/renderer/light.nim:9-17). */
enum rt_light_type { RT_DISTANT_LIGHT = 0, RT_POINT_LIGHT = 1 };

/* AntialiasKind (src/renderer/renderer.nim:11-12). */
/* Antialias kinds (renderer.nim:14-21 AntialiasKind). The stochastic kinds
 * (sampling.nim:21-113) draw from a counter-based RNG keyed by
 * (rt_options.seed, absolute pixel, draw index) instead of the reference's
 * clock-seeded Nim `random` — reproducible, and independent of how rows are
 * split across calls, bands or GPUs. float32: (correlated) multi-jittered up
 * to grid_size 32; float64: up to 256. */
enum rt_aa_kind {
  RT_AA_NONE = 0,
  RT_AA_GRID = 1,
  RT_AA_JITTERED = 2,
  RT_AA_MULTI_JITTERED = 3,
  RT_AA_CORRELATED_MULTI_JITTERED = 4
};

/* Arithmetic precision of the device path. RT_FP64 repeats the reference's
 * float64 arithmetic operation for operation (parity mode); RT_FP32 is the
 * performance mode (parity within the tolerance stated in DESIGN.md). */
enum rt_precision { RT_FP32 = 0, RT_FP64 = 1 };

/* TriangleMesh data (src/renderer/geom.nim:151-155, src/loaders/obj.nim:87-126).
 * Face i uses vertices faces[3i..3i+2]; its normal is normals[3i..3i+2]
 * (one normal per face, obj.nim:65-84). normals == NULL means "compute as
 * obj.nim calcNormals does": normalize(cross(v1 - v0, v2 - v0)). */
typedef struct rt_mesh_desc {
  const double *vertices;  /* num_vertices * 3 (x, y, z), object space */
  int64_t num_vertices;
  const int32_t *faces;    /* num_faces * 3 zero-based vertex indices   */
  int64_t num_faces;
  const double *normals;   /* num_faces * 3, or NULL                    */
} rt_mesh_desc;

/* Object{geometry, material} (src/renderer/scene.nim:6-9,
 * src/renderer/material.nim:4-7). world_to_object is the caller's
 * objectToWorld.inverse (geom.nim:159-198), passed through unchanged so that
 * host and device use identical matrices. */
typedef struct rt_object_desc {
  int32_t type;                /* rt_geom_type                           */
  int32_t mesh;                /* RT_MESH: index into rt_scene_desc.meshes */
  double object_to_world[16];
  double world_to_object[16];
  double radius;               /* RT_SPHERE: Sphere.r                    */
  double box_min[3];           /* RT_BOX: aabb.vmin (object space)       */
  double box_max[3];           /* RT_BOX: aabb.vmax                      */
  double albedo[3];            /* Material.albedo                        */
  double reflection;           /* Material.reflection                    */
} rt_object_desc;

typedef struct rt_light_desc {
  int32_t type;                /* rt_light_type                          */
  int32_t reserved;
  double color[3];
  double intensity;
  double dir[3];               /* DistantLight.dir (travel direction)    */
  double pos[3];               /* PointLight.pos                         */
} rt_light_desc;

/* Mesh BVH builder. Either tree gives the brute-force answer (closest t,
 * lowest face index on ties), so images and Stats do not depend on it. */
typedef enum rt_bvh_builder {
  RT_BVH_SAH = 0,  /* host binned SAH (32 bins, leaves <= 4 faces): best tracing */
  RT_BVH_PLOC = 1  /* on the device: Morton sort + PLOC clustering + SAH leaf
                      collapse, same node format; ~100x faster to build      */
} rt_bvh_builder;

/* Scene (src/renderer/scene.nim:11-18). */
typedef struct rt_scene_desc {
  const rt_object_desc *objects;
  int32_t num_objects;
  int32_t num_lights;
  const rt_light_desc *lights;
  const rt_mesh_desc *meshes;
  int32_t num_meshes;
  int32_t bvh_builder;         /* rt_bvh_builder (0 = host binned SAH)    */
  double fov;                  /* degrees, Scene.fov                     */
  double camera_to_world[16];  /* Scene.cameraToWorld                    */
  double bg_color[3];          /* Scene.bgColor                          */
} rt_scene_desc;

/* Options (src/renderer/renderer.nim:24-28) plus the device-path knobs. */
typedef struct rt_options {
  int32_t width, height;       /* Options.width/height                   */
  int32_t aa_kind;             /* Options.antialias.kind (rt_aa_kind)    */
  int32_t grid_size;           /* Options.antialias.gridSize (m)         */
  double bias;                 /* Options.bias                           */
  int32_t max_ray_depth;       /* Options.maxRayDepth                    */
  int32_t precision;           /* rt_precision                           */
  uint64_t seed;               /* stochastic samplers: counter-RNG seed  */
  uint32_t flags;              /* RT_FLAG_*                              */
  uint32_t reserved;
} rt_options;

/* Accepted for compatibility and ignored: shadow rays always stop searching
 * a mesh once the reference's outcome and hit count are decided (an exact
 * early exit: image and Stats identical to the closest-hit reference). */
#define RT_FLAG_ANYHIT_SHADOWS 0x1u
/* Run the instrumented kernel that also counts BVH node / triangle record
 * fetches (rt_scene_last_counters). Slower; the image and Stats are the same. */
#define RT_FLAG_COUNT_TRAVERSAL 0x2u
/* float32 kernel: always hand pixel groups out in screen order. By default a
 * short launch (a band set of a multi-GPU frame) that repeats a mapping already
 * rendered on this scene hands them out longest-first, from per-group
 * durations measured on its first launch. Scheduling only: the image and
 * Stats are the same either way. */
#define RT_FLAG_NO_REORDER 0x4u
/* float32 kernel: search the mesh BVH for every ray. By default camera rays
 * (>= 16 samples per pixel) and shadow rays to distant lights of a scene with
 * one mesh object search the faces binned for their pixel / light-grid cell
 * instead. The image and Stats are the same either way. */
#define RT_FLAG_NO_BINNING 0x8u
/* float32 kernel: render every pixel group with the one general kernel. By
 * default a launch whose pixel records mark pixels lean (no camera ray can hit
 * the scene's mesh and every light is a distant light whose shadow rays
 * provably miss it) renders those pixels with a second, lean-only kernel from
 * a per-launch list. Scheduling only: the image and Stats are the same. */
#define RT_FLAG_NO_SPLIT 0x10u
/* float32 kernel, two-class launches: render the general (not lean) pixels
 * with the one-sample loop of the general kernel. By default, in scenes of
 * one mesh object with distant lights only and no reflection, they render in
 * a kernel that carries several samples per lane through each face list
 * (falling back to the one-sample loop for a pixel whose shadow rays need
 * the BVH). Scheduling only: the image and Stats are the same. */
#define RT_FLAG_NO_BATCH 0x20u
/* Test hook: the batched general kernel discards each general pixel's
 * batches at its last one and re-renders the pixel with the one-sample loop
 * (the path it takes when a shadow ray needs the BVH). Same image and Stats. */
#define RT_FLAG_BATCH_FALLBACK 0x40u
/* float32 kernel, two-class launches: render lean pixels with the general
 * lean kernel. By default, in scenes whose only analytic object is one
 * translated plane (a mesh on a ground plane) with one or two distant lights
 * and akGrid sampling of m | 64 with spp a multiple of 256, they render in a
 * kernel specialised for that case. Scheduling only: same image and Stats. */
#define RT_FLAG_NO_LEAN1 0x80u
/* float32 kernel, two-class launches in the same one-plane scenes: render the
 * general pixels with the general batched kernel instead of the one
 * specialised for them. Scheduling only: same image and Stats. */
#define RT_FLAG_NO_GEN1 0x100u
/* _device calls with out == NULL: the caller will not read this call's Stats
 * (rt_scene_last_stats then fails), so the per-call Stats reduction is not
 * launched — the render kernels are all the call puts on the stream. Ignored
 * when out != NULL or with RT_FLAG_COUNT_TRAVERSAL. */
#define RT_FLAG_NO_STATS 0x200u
/* float32 kernel, one-plane two-class launches: launch the general and the
 * lean pixels' kernels separately. By default both lists run in one merged
 * kernel (general items first, then lean ones). Same image and Stats. */
#define RT_FLAG_NO_MIX 0x400u
/* Record HIP events (on the call's stream) around the call's two parts: the
 * camera-dependent data it builds on the device (camera-ray face lists, pixel
 * records, lean / general lists, object masks) and its render kernels;
 * rt_scene_last_timing reads them. Same image and Stats. */
#define RT_FLAG_TIMING 0x800u
/* float32 kernel, scenes of spheres / boxes / planes with distant lights and
 * no reflection: trace one sample per lane at a time. By default such pixels
 * carry 4 samples per lane through their object-binned object and light
 * loops (and a 64-spp frame uses 16 lanes per pixel to fill that batch).
 * Same image and Stats. */
#define RT_FLAG_NO_OBJ_BATCH 0x1000u
/* float32 kernel, scenes with reflective materials: queue the reflected rays
 * per wave and trace them in full 64-ray passes (k_render_wave), the pixel's
 * deeper levels summed in 32.32 fixed point — the image differs from the
 * default by float rounding only, the Stats are the same. By default each
 * reflected ray is traced in the lane of its camera sample, one level after
 * another: measured faster on the scenes here, whose reflected rays stay
 * coherent within a wave (DESIGN.md "Reflection-ray compaction"). */
#define RT_FLAG_COMPACT 0x2000u
/* float64 (parity) mode: render with one lane per pixel and the BVH for every
 * ray the pixel records do not rule out. By default akGrid frames of >= 64
 * samples per pixel render one pixel per wave (64 samples side by side; the
 * camera rays search the pixel's face list and the shadow rays to distant
 * lights their light-grid cells), each pixel's samples still summed in sample
 * order. The image and Stats are the same, bit for bit. */
#define RT_FLAG_F64_PER_LANE 0x4000u

/* Stats (src/renderer/stats.nim:4-13) plus ray counts for Mray/s. */
typedef struct rt_stats {
  uint64_t num_primary_rays;        /* renderer.nim:138,155             */
  uint64_t num_intersection_tests;  /* renderer.nim:58                  */
  uint64_t num_intersection_hits;   /* renderer.nim:65                  */
  uint64_t num_shadow_rays;         /* one per light per shaded hit     */
  uint64_t num_reflection_rays;     /* renderer.nim:114-118             */
} rt_stats;

/* Device-side work counters of the last render (algorithmic traffic). */
typedef struct rt_traversal_counters {
  uint64_t wave_node_fetches;  /* BVH node records fetched (per wave)     */
  uint64_t wave_tri_fetches;   /* triangle records fetched (per wave)     */
  uint64_t lane_node_visits;   /* sum over rays of node records visited
                                  (a ray visits a node whose box it hit)  */
  uint64_t lane_tri_tests;     /* sum over rays of triangle tests         */
} rt_traversal_counters;

typedef struct rt_scene_info {
  int64_t num_objects, num_lights, num_meshes;
  int64_t num_triangles;       /* all meshes                             */
  int64_t num_bvh_nodes;       /* all meshes                             */
  int32_t max_bvh_depth;
  int32_t device;
  int64_t device_bytes;        /* scene bytes in HBM: geometry, BVH, bins and the per-call buffer sets */
  double build_ms;             /* host BVH build + upload wall time      */
} rt_scene_info;

typedef struct rt_scene rt_scene; /* opaque, owns device buffers */

/* ---- library ----------------------------------------------------------- */

/* ABI version of the loaded library (RTMI_ABI_VERSION). */
int rt_version(void);

/* Hash of the native sources the library was built from (16 hex digits:
 * sha256 of csrc/, the Makefile and this header, nim-raytracer_amd/rtmi/
 * srchash.py): build provenance for benchmarks and profiles. */
const char *rt_build_source_hash(void);

/* Message of the last failed call on this thread ("" if none). */
const char *rt_last_error(void);

/* initRenderer* (renderer.nim:214-215) equivalent: bind the calling thread
 * to HIP device `device` and check it is a gfx950 GPU. Safe to call again. */
int rt_init(int device);

/* Number of visible GPUs (0 when none; never fails). */
int rt_device_count(void);

/* ---- scene ------------------------------------------------------------- */

/* Flatten, build the per-mesh BVH and upload everything to the current
 * device. desc and all arrays it points to may be freed after return. */
int rt_scene_create(const rt_scene_desc *desc, rt_scene **out_scene);
/* Waits for a call still running on the scene in another thread, then frees
 * it. No call may START on a scene once its destroy has begun (the caller's
 * own bookkeeping: INTEGRATION.md's binding retires a replaced scene only
 * after its in-flight renderLine calls have returned). */
int rt_scene_destroy(rt_scene *scene);
int rt_scene_get_info(const rt_scene *scene, rt_scene_info *out);

/* Replace the scene's camera: Scene.cameraToWorld (column-major, glm) and
 * Scene.fov in degrees (scene.nim:14-16), which renderLine re-reads on every
 * call (renderer.nim:135-136, 150-153 via castPrimaryRay :31-44). Takes
 * effect from the next render call; the geometry, BVH and light grids are
 * kept (every camera-dependent structure is rebuilt by each render call
 * anyway). Waits for the scene's earlier calls. RT_E_INVALID for a non-finite
 * matrix or a fov outside (0, 180). */
int rt_scene_set_camera(rt_scene *scene, const double camera_to_world[16],
                        double fov_deg);

/* ---- rendering ----------------------------------------------------------
 * All render calls implement renderLine (renderer.nim:162-211) for every row
 * y in countup(y0, y1 - 1, step):
 *   for x in countup(0, width - 1, step):
 *     if step < maxStep and (x and (2*step-1)) == 0 and (y and (2*step-1)) == 0:
 *       continue                      # already rendered at a coarser level
 *     color = calcPixel(...)          # akNone: 1 sample at (x, y); akGrid: m*m
 *     fill fb[x..x+step-1, y..y+step-1] (clipped) with color
 * step and max_step must be powers of two with max_step >= step.
 * `out` receives the summed Stats of the call (may be NULL for the _device
 * forms, which then do not synchronise the stream).
 * The per-call camera-dependent build has no capacity failure: a pixel
 * whose face list outgrows its slots keeps its true length and its camera
 * rays take the BVH (the same answers).
 */

/* Host framebuffer form: fb_rgb is caller memory of fb_w*fb_h*3 floats with
 * fb_w == opts->width and fb_h == opts->height. Thread-safe: concurrent
 * callers on disjoint rows are serialised internally (renderLine is called
 * concurrently by the reference's pool, workerpool.nim:172-223). */
int rt_render_lines(rt_scene *scene, const rt_options *opts, float *fb_rgb,
                    int32_t fb_w, int32_t fb_h, int32_t y0, int32_t y1,
                    int32_t step, int32_t max_step, rt_stats *out);

/* Device framebuffer form (the fast path: whole frame, nothing crosses
 * PCIe). d_fb is a device pointer to width*height*3 floats. */
int rt_render_lines_device(rt_scene *scene, const rt_options *opts,
                           float *d_fb, int32_t y0, int32_t y1, int32_t step,
                           int32_t max_step, void *hip_stream, rt_stats *out);

/* Multi-GPU shard: image rows are cut into bands of band_h rows; band b is
 * owned by rank b % world. Renders this rank's bands (step 1) into the
 * compact device buffer d_bands laid out as
 *   [ceil(ceil(height/band_h)/world) * band_h rows][width][3] float32,
 * i.e. local band k occupies rows [k*band_h, (k+1)*band_h). Rows past the
 * image bottom are left untouched. */
int rt_render_bands_device(rt_scene *scene, const rt_options *opts,
                           float *d_bands, int32_t band_h, int32_t rank,
                           int32_t world, void *hip_stream, rt_stats *out);

/* Rank-0 epilogue of the framebuffer gather: d_gathered holds `world`
 * compact band buffers back to back (an all-gather of rt_render_bands_device
 * outputs); writes the interleaved image to d_fb (width*height*3). */
int rt_unshard_bands_device(const float *d_gathered, float *d_fb,
                            int32_t width, int32_t height, int32_t band_h,
                            int32_t world, void *hip_stream);

/* Rows per rank-local compact band buffer (helper for sizing d_bands). */
int rt_band_rows(int32_t height, int32_t band_h, int32_t world,
                 int32_t *out_rows);

/* Stats of the last render call on this scene (waits for it): for
 * asynchronous _device calls made with out == NULL (RT_E_INVALID if that
 * call set RT_FLAG_NO_STATS). */
int rt_scene_last_stats(rt_scene *scene, rt_stats *out);

/* Durations of the last call made with RT_FLAG_TIMING (waits for it): its
 * per-call camera-dependent build and its render kernels (incl. the Stats
 * reduction), in milliseconds. RT_E_INVALID if that call did not set the flag. */
int rt_scene_last_timing(rt_scene *scene, double *setup_ms, double *render_ms);

/* ---- one process, several GPUs (SURVEY.md 8(b) rt_render_frame_multi) ---- */

/* The scene replicated on every listed device (a device may repeat: several
 * ranks on one GPU); rows cut into band_h-row bands dealt round-robin
 * (band b -> rank b % num_devices; band_h 0 means 4); every rank renders its
 * bands on its own device at the same time, the compact band buffers move to
 * devices[0] over xGMI (peer copies) and are un-interleaved there. Images and
 * Stats equal the single-device frame. For one process per GPU use
 * rt_render_bands_device + rt_unshard_bands_device with RCCL instead. */
typedef struct rt_multi rt_multi;
int rt_multi_create(const rt_scene_desc *desc, const int32_t *devices,
                    int32_t num_devices, int32_t band_h, rt_multi **out);
/* Whole frame (step 1) into d_fb, a width*height*3 float32 buffer on
 * devices[0]; out != NULL waits for the frame and sums the Stats. */
int rt_render_frame_multi_device(rt_multi *m, const rt_options *opts,
                                 float *d_fb, rt_stats *out);
/* Whole frame into the caller's host framebuffer (fb_w*fb_h*3 floats). */
int rt_render_frame_multi(rt_multi *m, const rt_options *opts, float *fb,
                          int32_t fb_w, int32_t fb_h, rt_stats *out);
/* rt_scene_set_camera on every rank's scene. */
int rt_multi_set_camera(rt_multi *m, const double camera_to_world[16],
                        double fov_deg);
int rt_multi_destroy(rt_multi *m);

/* ---- render queue (workerpool.nim WorkerPool[WorkMsg, ResponseMsg]) ---- */

/* The pool raytracer.nim and gui.nim drive (src/concurrency/workerpool.nim;
 * WorkMsg / ResponseMsg, src/raytracer.nim:13-32; gui.nim:98-122,206-280),
 * over the GPU: one host thread per queue takes the longest run of queued
 * lines that share options, framebuffer, step and max_step and follow each
 * other at `step`, and renders it with ONE rt_render_lines call (one launch
 * per refinement level when the caller queues a whole level, as gui.nim
 * does). Every message gets its own response, in queue order; a run's Stats
 * ride on its last line's response, the others carry zero Stats (callers sum
 * them). States and return values follow workerpool.nim; every command has
 * completed when it returns, so the queue is always ready (isReady). The
 * queue must be destroyed before its scene. */
typedef struct rt_queue rt_queue;

typedef enum rt_queue_state_kind {
  RT_QUEUE_STOPPED = 0, /* wsStopped: work is queued, not started */
  RT_QUEUE_RUNNING = 1, /* wsRunning                             */
  RT_QUEUE_SHUTDOWN = 2 /* wsShutdown: no more work accepted       */
} rt_queue_state_kind;

typedef struct rt_response { /* ResponseMsg (raytracer.nim:21-23) + the line */
  int32_t line;
  int32_t status;            /* RT_OK, or the render call's error code    */
  rt_stats stats;
  char error[128];           /* rt_last_error() text when status != 0     */
} rt_response;

/* initRenderWorkers (raytracer.nim:35-38); starts stopped. */
int rt_queue_create(rt_scene *scene, rt_queue **out);
/* start / stop (workerpool.nim:253-275): 1 done, 0 not in the required
 * state (stopped / running). stop lets the batch in flight finish and
 * keeps queued lines queued. */
int rt_queue_start(rt_queue *q);
int rt_queue_stop(rt_queue *q);
int rt_queue_state(rt_queue *q);    /* rt_queue_state_kind, or < 0 */
int rt_queue_is_ready(rt_queue *q); /* 1 */
/* queueWork (workerpool.nim:235): renderLine(line, step, maxStep) into the
 * caller's host framebuffer fb (fb_w*fb_h*3 floats, written by the queue's
 * thread until the line's response arrives); step / max_step 0 mean 1
 * (raytracer.nim:26-27). */
int rt_queue_work(rt_queue *q, const rt_options *opts, float *fb,
                  int32_t fb_w, int32_t fb_h, int32_t line, int32_t step,
                  int32_t max_step);
/* tryRecvResult (workerpool.nim:240): 1 and *out filled, or 0 if no
 * response is waiting. A failed line's message is also set as this
 * thread's rt_last_error(). */
int rt_queue_try_recv(rt_queue *q, rt_response *out);
/* Lines queued or in flight. */
int rt_queue_pending(rt_queue *q);
/* reset (workerpool.nim:285-314): stop, drop queued work and undelivered
 * responses; 1 done, 0 after shutdown. */
int rt_queue_reset(rt_queue *q);
/* shutdown (workerpool.nim:359): 1 done, 0 if already shut down. */
int rt_queue_shutdown(rt_queue *q);
/* close (workerpool.nim:371) + free, from any state. */
int rt_queue_destroy(rt_queue *q);

/* ---- output (framebuf.nim:55-93 writePpm) ------------------------------ */

/* The P6 payload of writePpm for a device framebuffer (width*height*3
 * float32, the Framebuf.data layout): per component clamp to [0, 1], optional
 * linearToSRGB (color.nim:17-22), round(c * (2^bits - 1)); bits in 1..16;
 * bits <= 8: one byte per component, else two bytes big-endian. d_out
 * receives rt_ppm_payload_bytes() bytes (device memory). Replaces
 * framebuf.nim:82-88's per-component loop; the caller writes
 * rt_ppm_header() and then the payload. */
int rt_ppm_encode_device(const float *d_fb, int32_t width, int32_t height,
                         int32_t bits, int32_t srgb, void *d_out,
                         void *hip_stream);
/* Payload size in bytes (width*height*3*(bits <= 8 ? 1 : 2)), or < 0. */
int64_t rt_ppm_payload_bytes(int32_t width, int32_t height, int32_t bits);
/* writeHeader (framebuf.nim:60-61): "P6 <w> <h> <maxval> " into buf; returns
 * its length (excluding the NUL), or < 0 if buf_len is too small. */
int rt_ppm_header(int32_t width, int32_t height, int32_t bits, char *buf,
                  int32_t buf_len);

/* ImageRGBA.copyFrom (src/utils/image.nim:45-54) as a GPU post-pass: the
 * width*height*3 float32 device framebuffer -> width*height RGBA8 pixels at
 * d_out (device memory, 4-B aligned), round(c * 0xff).uint8 per component
 * and `alpha`, for the GUI's texture upload without a float32 round trip.
 * No clamp, like the reference: components outside [0, 255] after rounding
 * keep the low 8 bits of the x86-64 int32 conversion (the reference's
 * release build). Asynchronous on `stream`. */
int rt_rgba_encode_device(const float *d_fb, int32_t width, int32_t height,
                          uint8_t alpha, void *d_out, void *stream);

/* Traversal counters of the last render call on this scene (waits for it).
 * Zero unless that call set RT_FLAG_COUNT_TRAVERSAL. */
int rt_scene_last_counters(rt_scene *scene, rt_traversal_counters *out);

/* Work split of the last render call on this scene: pixel groups rendered by
 * the lean-pixel kernel and by the general kernel (RT_FLAG_NO_SPLIT; a
 * float64 call counts every group as general). Host-side bookkeeping, no wait. */
int rt_scene_last_split(rt_scene *scene, int64_t *lean_groups, int64_t *general_groups);
/* Of the last render call's general pixel groups: how many went to the
 * batched general kernel (0 with RT_FLAG_NO_BATCH or where it does not
 * apply), and how many of those it re-rendered with the one-sample loop
 * because a shadow ray needed the BVH (as of the last call that returned
 * Stats; -1 before any). Diagnostics for tests and the benchmark. */
int rt_scene_last_batch(rt_scene *scene, int64_t *batched_groups, int64_t *fallback_groups);
/* Which kernels rendered the last call's two classes: bits 0-1 the lean
 * pixels' (0 none — no two-class launch, 1 the general lean kernel, 2 the
 * one-plane lean kernel, RT_FLAG_NO_LEAN1), bits 2-3 the general pixels'
 * (0 the one-sample kernel, 1 the general batched kernel, 2 the one-plane
 * batched kernel, RT_FLAG_NO_GEN1); 3 in both: the merged one-plane kernel
 * (RT_FLAG_NO_MIX); bit 4: reflected rays compacted per wave (reflective
 * scenes, RT_FLAG_COMPACT); bits 8-15: lanes per lean pixel of a two-class
 * call (4 or 16 for the one-plane lean kernels, 64 for one pixel per wave;
 * 0 otherwise) — mask with 0x1f to compare the kernel kinds. Host-side
 * bookkeeping, no wait. */
int rt_scene_last_lean_kernel(rt_scene *scene, int32_t *kind);

/* ---- helpers ----------------------------------------------------------- */

/* glm-style inverse of a column-major 4x4 (what geom.nim's
 * objectToWorld.inverse computes); RT_E_INVALID if singular. */
int rt_mat4_inverse(const double m[16], double out[16]);

/* .geom triangle soup (format of test/test.nim:14-26 and the writer
 * src/loaders/objconv.nim:139-153): int32 N, then N*3 vertices of 3 float32.
 * Query form: pass vertices == NULL to get *num_triangles only; then pass a
 * buffer of num_triangles*9 doubles. */
int rt_load_geom(const char *path, int64_t *num_triangles, double *vertices);

/* OBJ reader of src/loaders/obj.nim:87-126: "v x y z" and "f a b c" lines
 * (1-based indices; a 4th face vertex is ignored), other lines skipped;
 * tokens that do not parse entirely leave 0 (a coordinate) or index 0 (a
 * face vertex), as the reference's try/except defaults do — so "f 1//2 ..."
 * gives index 0 unless RT_OBJ_SLASH_INDICES takes the integer before the
 * first '/'. Face normals are not read (the reference computes them:
 * calcNormals, done by rt_scene_create when rt_mesh_desc.normals is NULL).
 * Query form: vertices == faces == NULL sets the two counts; then pass
 * buffers of num_vertices*3 doubles and num_faces*3 int32 (0-based). */
#define RT_OBJ_SLASH_INDICES 0x1u
int rt_load_obj(const char *path, uint32_t flags, int64_t *num_vertices,
                double *vertices, int64_t *num_faces, int32_t *faces);

/* objconv's writeGeom (src/loaders/objconv.nim:139-153): int32 face count,
 * then each face's three vertices as float32 x, y, z. */
int rt_write_geom(const char *path, const double *vertices,
                  int64_t num_vertices, const int32_t *faces,
                  int64_t num_faces);

#ifdef __cplusplus
}
#endif

#endif /* RTMI_H */
