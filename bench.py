#!/usr/bin/env python3
"""Benchmark: Mray/s (primary + shadow) on bunny.geom, 1920x1080, 256 spp.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

One step = one full frame of BASELINE config C3 (mesh-bunny layout: baked
bunny.geom 69,451 triangles + ground plane, 2 distant lights, akGrid 16x16 =
256 samples per pixel, fp32 performance mode) rendered from a scene resident
in HBM into a device framebuffer. Every step does the whole frame's work:
the render call builds its camera-dependent data on the device (camera-ray
face lists, pixel records with the shadow skip bits, the lean / general
lists — rt_frame.h) and then traces every ray it counts; nothing that
depends on the camera is kept between steps. What is built once per scene
(BVH, light grids) depends on the geometry and the lights only.

N = 1: one whole-frame call per step. N > 1 (torchrun): the same frame cut
into 4-row bands dealt round-robin to the ranks; each rank builds and renders
its own bands, one RCCL gather + an on-GPU un-interleave assembles the frame
on rank 0 (strong scaling; every gather inside the timed region, frame k's
overlapping frame k+1's render from a second band buffer).

Printed (rank 0, one JSON line): value = (primary + shadow rays of all ranks)
x K / max-over-ranks wall time, plus
  roofline     — the render kernels of the call (C3-C5: the merged kernel
                 k_render_mix1), timed with HIP events inside the library
                 (RT_FLAG_TIMING, the call's stream) in a pass after the
                 timed region. The kernels are instruction-issue bound
                 (wave-uniform scalar record fetches serve 64 lanes; the
                 records live in the caches): bound "issue", achieved = wave64
                 VALU instructions per second (PMC SQ_INSTS_VALU of the same
                 kernels, profiles/pmc_summary.json, used only when its source
                 hash matches these sources) against 1024 SIMDs x 2.4 GHz / 2
                 cycles; HBM bytes per call from the same summary beside it;
  cpu_baseline — the fp64 oracle (the reference algorithm: linear objects,
                 brute-force mesh, scanline thread pool) on this host, 1 spp on
                 a bounded row subsample of the same frame (rank 0, N = 1 only).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "nim-raytracer_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md "Chip-level parameters")
# SURVEY.md 8(d) algorithmic bytes per ray: 32 B per BVH box tested (a node
# record visited = its two child boxes = 64 B), 36 B per triangle tested (three
# fp32 vertices, the .geom record), 12 B per pixel written (12/spp per ray)
SURVEY_BOX_BYTES = 32
SURVEY_TRI_BYTES = 36
PIXEL_BYTES = 12
BAND_H = 4             # rows per band (round-robin over ranks)


def _scene(name):
    from rtmi import scenes
    return {"bunny": scenes.mesh_bunny, "boxes2": scenes.boxes2, "torus": scenes.torus_scene,
            "mix": scenes.mesh_mix}[name]()


# BASELINE.json configs on one GPU (C4/C5 are quoted on 8 GPUs; at N=1 this is
# one GPU's whole frame, at N>1 the band-sharded frame)
CONFIGS = {
    "C2": ("boxes2", 1920, 1080, 8, "C2: boxes2.nim (16 analytic primitives, 1 distant light)"),
    "C3": ("bunny", 1920, 1080, 16, "C3: bunny.geom baked x30 + ground plane, mesh-bunny.nim lights/camera"),
    "C4": ("bunny", 3840, 2160, 32, "C4: bunny.geom baked x30 + ground plane, mesh-bunny.nim lights/camera"),
    "C5": ("torus", 3840, 2160, 64, "C5: 1,000,000-triangle procedural torus + ground, mesh-bunny.nim lights/camera"),
    # not a BASELINE config: a scene outside the list envelope (a reflective
    # mesh, a point light, analytic objects around it), so every ray of it
    # takes the wave-coherent BVH traversal (k_render_fast) — that path's line
    "BVHMIX": ("mix", 1920, 1080, 8, "mesh-mix: reflective mesh between spheres/boxes, point + distant light "
                                     "(the BVH path: k_render_fast)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C3", choices=sorted(CONFIGS),
                    help="BASELINE.json config (C3 = the headline metric)")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--grid", type=int, default=None, help="akGrid m (spp = m*m)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the fp64_parity / bvh_path sub-measurements after the timed region")
    ap.add_argument("--bvh", default="sah", choices=["sah", "ploc"],
                    help="mesh BVH builder: host binned SAH (default) or device PLOC")
    ap.add_argument("--flags", type=int, default=0, help="rt_options.flags (1 = any-hit shadows)")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "fp64"],
                    help="fp32 = the performance kernels (the headline); fp64 = the parity mode the Nim "
                         "binding defaults to (bit-exact against the oracle): the cost of exactness")
    return ap.parse_args()


def cpu_baseline(scene, width, height, target_s, bvh=False):
    """The oracle (reference algorithm, fp64; bvh=False: the reference's
    brute-force mesh loop, bvh=True: the same answers from a per-ray BVH) on
    a uniform row subsample of the same frame at 1 spp, on this host's cores."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    from rtmi import Antialias, Options, Precision, akGrid

    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    threads = max(1, min(16, ncpu))  # the GPU box's CPU share is 16 threads
    opts = Options(width=width, height=height, antialias=Antialias(akGrid, 1), bias=1e-4,
                   precision=Precision.fp64)
    osc = oracle.OracleScene(scene, bvh=bvh)
    # calibrate on a sparse probe, then size the sample to ~target_s: a row
    # subsample at 1 spp, or (a fast CPU path) the whole frame at m x m spp
    probe = list(range(7, height, max(1, height // 24)))
    _, st, secs = osc.render(opts, rows=probe, nthreads=threads)
    per_row = secs / len(probe)
    n = int(max(len(probe), min(height, target_s / max(per_row, 1e-6))))
    grid = 1
    if n >= height:
        grid = max(1, min(16, int((target_s / max(per_row * height, 1e-6)) ** 0.5)))
        opts = Options(width=width, height=height, antialias=Antialias(akGrid, grid), bias=1e-4,
                       precision=Precision.fp64)
    stride = max(1, height // n)
    rows = list(range(stride // 2, height, stride))
    _, st, secs = osc.render(opts, rows=rows, nthreads=threads)
    if n >= height and grid < 16 and secs < target_s / 3:  # one refinement of the sample size
        grid = max(grid, min(16, int(grid * (target_s / max(secs, 1e-6)) ** 0.5)))
        opts = Options(width=width, height=height, antialias=Antialias(akGrid, grid), bias=1e-4,
                       precision=Precision.fp64)
        _, st, secs = osc.render(opts, rows=rows, nthreads=threads)
    rays = st.numPrimaryRays + st.numShadowRays
    return {
        "value": rays / secs / 1e6,
        "unit": "Mray/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"oracle/rt_oracle.c (fp64 restatement of the reference path: linear object loop, "
                   + ("per-ray fp64 binned-SAH BVH with the brute-force loop's exact answers"
                      if bvh else "brute-force TriangleMesh.intersect")
                   + f", scanline pool of {threads} threads), same scene/camera at {grid * grid} spp "
                   f"(akGrid {grid}), "
                   f"{len(rows)} of {height} rows (every {stride}th), {rays} rays in {secs:.2f} s"),
    }


SIMDS = 1024           # MI355X: 256 CUs x 4 SIMDs (MI355X_MICROARCH.md)
CUS = 256
CLOCK_GHZ = 2.4        # peak engine clock
VALU_CYCLES = 2        # a wave64 VALU instruction issues over 2 cycles per SIMD (MI355X_MICROARCH.md)
VALU_PEAK_GINST = SIMDS * CLOCK_GHZ / VALU_CYCLES   # 1228.8 G wave64 VALU instructions / s
SALU_PEAK_GINST = CUS * CLOCK_GHZ                   # one scalar unit per CU, one instruction per cycle


F64_VALU_CYCLES = 4    # FP64 FMA/MUL/ADD/TRANS: half the FP32 rate (78.6 vs 157.3 TF spec) = 4 cycles per wave64
F64_COUNTERS = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64")


def issue_roofline(c, sec):
    """Issue-bound roofline of a render call from its per-call PMC counters
    `c` over `sec` seconds. When the F64 op counts are present the issue
    time is weighted: an F64 VALU instruction occupies its SIMD 4 cycles,
    every other VALU instruction 2 (MI355X_MICROARCH.md: 64 FP32 FLOP/clk/SIMD,
    FP64 at half that), and frac = issue cycles / (SIMDs x clock x sec)."""
    out = {}
    if "SQ_INSTS_VALU" not in c:
        return out
    ach = c["SQ_INSTS_VALU"] / sec / 1e9
    out["achieved"] = round(ach, 1)
    out["frac"] = round(ach / VALU_PEAK_GINST, 4)
    if all(k in c for k in F64_COUNTERS):
        f64 = sum(c[k] for k in F64_COUNTERS)
        cycles = (c["SQ_INSTS_VALU"] - f64) * VALU_CYCLES + f64 * F64_VALU_CYCLES
        out["f64_valu_share"] = round(f64 / c["SQ_INSTS_VALU"], 4)
        out["frac_f64_weighted"] = round(cycles / (SIMDS * CLOCK_GHZ * 1e9 * sec), 4)
        out["f64_definition"] = ("frac_f64_weighted = (2 x non-F64 VALU + 4 x F64 VALU instructions, PMC "
                                 "SQ_INSTS_VALU and SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64) / (1024 SIMDs x "
                                 f"{CLOCK_GHZ} GHz x kernel time): the SIMD issue cycles the F64 mix needs")
    if "SQ_INSTS_SALU" in c:
        out["salu_frac"] = round(c["SQ_INSTS_SALU"] / sec / 1e9 / SALU_PEAK_GINST, 4)
    return out


def sub_measure(ds, opts, fb, stream, steps, warmup, key):
    """Time `steps` whole-frame calls of `opts` after `warmup` (barrier +
    synchronize around them, one event pair on the call stream), then one
    RT_FLAG_TIMING pass for the render kernels' time; PMC roofline from the
    committed summary under `key` when its sources match."""
    import dataclasses

    import torch

    from rtmi.abi import RT_FLAG_TIMING
    st = ds.render_device(opts, fb, stream=stream, stats=True)
    for _ in range(warmup):
        ds.render_device(opts, fb, stream=stream, stats=False)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        ds.render_device(opts, fb, stream=stream, stats=False)
    ev1.record(stream)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    topts = dataclasses.replace(opts, flags=opts.flags | RT_FLAG_TIMING)
    rms = []
    for _ in range(steps):
        ds.render_device(topts, fb, stream=stream, stats=False)
        rms.append(ds.last_timing()[1])
    render_ms = sum(rms) / len(rms)
    rays = st.numPrimaryRays + st.numShadowRays
    out = {"value": round(rays * steps / el / 1e6, 2), "unit": "Mray/s", "steps": steps, "warmup": warmup,
           "ms_per_step": round(el / steps * 1e3, 3), "call_ms": round(ev0.elapsed_time(ev1) / steps, 4),
           "kernel_ms": round(render_ms, 4), "primary_rays_per_frame": st.numPrimaryRays,
           "shadow_rays_per_frame": st.numShadowRays}
    pmc = load_pmc(key)
    if pmc is not None:
        c = pmc["counters_mean_per_dispatch"]
        sec = render_ms * 1e-3
        roof = issue_roofline(c, sec)
        if key.endswith("_fp64"):
            add_net_of_spills(roof, "k_render_px64ILi4ELi1E")
        if "hbm_bytes_per_launch" in pmc:
            roof["traffic"] = int(pmc["hbm_bytes_per_launch"])
            roof["hbm_gbs"] = round(pmc["hbm_bytes_per_launch"] / sec / 1e9, 1)
            roof["hbm_frac"] = round(pmc["hbm_bytes_per_launch"] / sec / 1e9 / HBM_PEAK_GBS, 4)
        roof["pmc"] = f"profiles/pmc_summary.json[{key}] (sources {pmc['source_hash']})"
        out["roofline"] = roof
    else:
        out["roofline"] = {"pmc": f"no PMC summary [{key}] for these native sources"}
    return out


def load_spill_share(kernel_pat):
    """profiles/spill_share.json (tools/spill_share.py) for these sources:
    the estimated share of a kernel's VALU instructions that are SGPR-spill
    lane moves, or None."""
    from rtmi._lib import kernel_source_hash
    try:
        with open(os.path.join(REPO, "profiles", "spill_share.json")) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("source_hash") != kernel_source_hash():
        return None
    return d.get("kernels", {}).get(kernel_pat)


def add_net_of_spills(roof, kernel_pat):
    """frac net of the kernel's SGPR-spill VALU: the static
    share and the loop-depth-weighted estimate (4 trips per loop level, an
    upper bound for the hot loops' trip counts)."""
    sp = load_spill_share(kernel_pat)
    if sp is None or roof.get("frac") is None:
        return
    w = sp["weighted_share_4_per_level"]
    roof["spill_valu_share_static"] = sp["static_share"]
    roof["spill_valu_share_est"] = w
    roof["frac_net_of_spills_est"] = round(roof["frac"] * (1.0 - w), 4)
    if "frac_f64_weighted" in roof:
        roof["frac_f64_weighted_net_of_spills_est"] = round(roof["frac_f64_weighted"] * (1.0 - w), 4)
    roof["spill_note"] = ("v_writelane/v_readlane (SGPR spills) share of the kernel's VALU: static count, and weighted "
                          "by 4 trips per loop level from the gfx950 assembly's loop depths (tools/spill_share.py, "
                          "profiles/spill_share.json)")


def load_pmc(workload_key):
    """Per-call PMC figures of the render kernels from the committed summary
    (profiles/pmc_summary.json, tools/pmc_summary.py) when it was measured on
    these native sources (never mix two builds), else None."""
    from rtmi._lib import kernel_source_hash
    p = os.path.join(REPO, "profiles", "pmc_summary.json")
    try:
        with open(p) as f:
            e = json.load(f).get(workload_key)
    except (OSError, ValueError):
        return None
    if e is None or e.get("source_hash") != kernel_source_hash():
        return None
    return e


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from rtmi import Antialias, Options, Precision, akGrid, scenes
    from rtmi._lib import kernel_source_hash, library_source_hash
    from rtmi.dist import band_rows, gather_bands
    from rtmi.renderer import DeviceScene

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    # launched by torchrun (even with one rank): the band + RCCL-gather path
    distributed = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ or "LOCAL_WORLD_SIZE" in os.environ
    # stdout carries exactly one JSON line: whatever else writes to fd 1 (the
    # RCCL banner at communicator creation) goes to stderr
    json_out = sys.stdout
    if distributed:
        sys.stdout.flush()
        json_out = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    scene_name, W, H, m, desc = CONFIGS[args.config]
    W = args.width or W
    H = args.height or H
    m = args.grid or m
    scene = _scene(scene_name)
    t0 = time.time()
    from rtmi.abi import RT_BVH_PLOC, RT_BVH_SAH
    ds = DeviceScene(scene, device=local, bvh_builder=RT_BVH_PLOC if args.bvh == "ploc" else RT_BVH_SAH)
    info = ds.info()
    setup_s = time.time() - t0
    fp64 = args.precision == "fp64"
    opts = Options(width=W, height=H, antialias=Antialias(akGrid, m), bias=1e-4,
                   precision=Precision.fp64 if fp64 else Precision.fp32, flags=args.flags)
    stream = torch.cuda.current_stream()
    # the first frame of this scene and image size also allocates the
    # per-call buffers and reads the camera-ray list size once (every frame
    # builds the lists themselves): timed on its own, beside the steps
    if not distributed:
        fb0 = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ds.render_device(opts, fb0, stream=stream, stats=False)
        torch.cuda.synchronize()
        first_frame_ms = (time.perf_counter() - t0) * 1e3
        del fb0
    else:
        first_frame_ms = None
    rows = band_rows(H, BAND_H, world)
    fb = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
    # two band buffers: frame k's gather (RCCL, its own stream) overlaps frame
    # k+1's render, which writes the other buffer
    local_bufs = [torch.zeros(rows * W * 3, dtype=torch.float32, device="cuda") for _ in range(2)]
    local_buf = local_bufs[0]
    gathered = torch.zeros(world * rows * W * 3, dtype=torch.float32, device="cuda")

    from rtmi.renderer import unshard_bands_device

    pending = [None]  # the previous frame's gather
    nframe = [0]

    def finish_frame():
        # complete the previous frame: its gather, then (rank 0) the
        # un-interleave into the frame buffer, in stream order (a side stream
        # for the un-interleave measured slower — it shares the 4 hardware
        # queues with the build and RCCL streams — and so did the stream-value
        # hand-off instead of events: DESIGN.md (e), round 6)
        if pending[0] is not None:
            pending[0].wait()
            pending[0] = None
            if rank == 0:
                unshard_bands_device(gathered, fb, W, H, BAND_H, world, stream=stream)

    def step(time_kernel=None):
        # render this rank's bands (world == 1: the whole frame, one band set)
        buf = local_bufs[nframe[0] % 2]
        nframe[0] += 1
        if time_kernel is not None and time_kernel[0] is not None:
            time_kernel[0].record(stream)
        if distributed:
            ds.render_bands_device(opts, buf, BAND_H, rank, world, stream=stream, stats=False)
        else:
            ds.render_device(opts, fb, stream=stream, stats=False)
        if time_kernel is not None and time_kernel[1] is not None:
            time_kernel[1].record(stream)
        if distributed:
            finish_frame()  # frame k-1, whose gather overlapped this render
            pending[0] = gather_bands(buf, gathered if rank == 0 else None, rows * W * 3, async_op=True)

    # warmup (+ the deterministic per-frame ray counts)
    from rtmi.abi import RT_FLAG_COUNT_TRAVERSAL, RT_FLAG_NO_BINNING, RT_FLAG_TIMING
    import dataclasses
    st = ds.render_bands_device(opts, local_buf, BAND_H, rank, world, stream=stream, stats=True)
    # SURVEY 8(d)'s per-ray BVH model (every ray traverses the scene BVH):
    # node visits / triangle tests of one instrumented launch of the BVH path
    # (k_render_fast<true>, RT_FLAG_COUNT_TRAVERSAL | RT_FLAG_NO_BINNING) —
    # a model of what a per-ray BVH tracer would read, not the timed kernels
    copts = dataclasses.replace(opts, flags=opts.flags | RT_FLAG_COUNT_TRAVERSAL | RT_FLAG_NO_BINNING,
                                precision=Precision.fp32)
    ds.render_bands_device(copts, local_buf, BAND_H, rank, world, stream=stream, stats=True)
    counters = ds.last_counters()
    for _ in range(max(0, args.warmup)):
        step()
    finish_frame()
    rays_local = st.numPrimaryRays + st.numShadowRays
    if distributed:
        t = torch.tensor([rays_local, st.numPrimaryRays, st.numShadowRays], dtype=torch.int64,
                         device="cuda")
        dist.all_reduce(t)
        rays_frame, prim_frame, shadow_frame = [int(x) for x in t.tolist()]
    else:
        rays_frame, prim_frame, shadow_frame = rays_local, st.numPrimaryRays, st.numShadowRays

    # timed region
    # one event pair around the K render calls (a timing event per step is
    # a marker packet between calls): call_ms = their GPU span / K
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step((ev0 if k == 0 else None, ev1 if k == args.steps - 1 else None))
    finish_frame()  # the last frame's gather + un-interleave, inside the timed region
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if distributed:
        e = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    call_ms = ev0.elapsed_time(ev1) / max(1, args.steps)
    lean_groups, general_groups = ds.last_split()
    kinds = ds.last_lean_kernel()
    lean_k = {0: None, 1: "k_render_lean", 2: "k_render_lean1q (one-plane lean pixels)", 3: None}[kinds & 3]
    gen_k = {0: "k_render_fast<false>", 1: "k_render_gen", 2: "k_render_gen1 (one-plane general pixels)",
             3: None}[kinds >> 2 & 3]
    kernel_desc = ("k_render_px64 (fp64 parity kernel: one pixel per wave, 64 samples side by side, camera rays "
                   "through the pixel's face list, shadow rays through their light-grid cells, samples summed in "
                   "sample order)" if fp64 else
                   "k_render_mix1 (one-plane scene: general pixels, then lean pixels, one merged kernel)"
                   if kinds == 15 else f"{gen_k} + {lean_k} (two-class launch)" if lean_k else gen_k)
    # after the timed region, the same steps once more with RT_FLAG_TIMING:
    # HIP events inside the library split each call into its per-call
    # camera-dependent build and its render kernels (each call waited for)
    topts = dataclasses.replace(opts, flags=opts.flags | RT_FLAG_TIMING)
    setup_ms, render_ms = [], []
    for _ in range(args.steps):
        ds.render_bands_device(topts, local_bufs[0], BAND_H, rank, world, stream=stream, stats=False)
        a_ms, b_ms = ds.last_timing()
        setup_ms.append(a_ms)
        render_ms.append(b_ms)
    setup_ms = sum(setup_ms) / len(setup_ms)
    render_ms = sum(render_ms) / len(render_ms)
    # after the timed region: frames that each follow a camera change
    # (rt_scene_set_camera, alternating two cameras 0.05 apart), so every call
    # also re-reads its list size and may grow the entry buffer — what an
    # interactive caller moving the camera every frame pays
    camera_change_ms = None
    if not distributed:
        from rtmi.glm import translate, vec3
        cams = [translate(scene.cameraToWorld, vec3(0.05, 0.0, 0.0)), scene.cameraToWorld]
        n_cam = max(4, args.steps)
        torch.cuda.synchronize()
        t_cam = time.perf_counter()
        for k in range(n_cam):
            ds.set_camera(cams[k % 2], scene.fov)
            ds.render_device(opts, fb, stream=stream, stats=False)
        torch.cuda.synchronize()
        camera_change_ms = (time.perf_counter() - t_cam) * 1e3 / n_cam
        ds.set_camera(scene.cameraToWorld, scene.fov)
    # outside the timed region: one more launch with Stats, for how many of
    # the batched general pixels fell back to the one-sample loop
    ds.render_bands_device(opts, local_bufs[0], BAND_H, rank, world, stream=stream, stats=True)
    batched_groups, batch_fallback = ds.last_batch()
    # outside the timed region: the gathered frame must equal one GPU's
    # single-call frame bit for bit (same samples, same arithmetic per pixel)
    frame_check = None
    if distributed and rank == 0:
        ref = torch.zeros_like(fb)
        ds.render_device(opts, ref, stream=stream, stats=False)
        torch.cuda.synchronize()
        frame_check = {"bit_identical_to_single_call_frame": bool(torch.equal(ref, fb))}

    # outside the timed region, one GPU only: the same frame in the parity
    # mode the Nim binding runs (float64, bit-exact against the oracle:
    # tests/test_gpu_px64.py::test_px64_full_c3_frame) and on the BVH path
    # that every scene outside the list envelope takes (RT_FLAG_NO_BINNING:
    # k_render_fast<false>, a per-ray wave-coherent BVH traversal for every
    # camera and shadow ray) — each timed like the headline, fewer steps
    extra = {}
    if not distributed and not fp64 and not args.flags and not args.no_extra and args.config in ("C2", "C3"):
        k_extra = max(2, min(args.steps, 5))
        base_key = f"{args.config.lower()}_{W}x{H}_m{m}_world{world}"
        o64 = dataclasses.replace(opts, precision=Precision.fp64)
        extra["fp64_parity"] = sub_measure(ds, o64, fb, stream, k_extra, 1, base_key + "_fp64")
        extra["fp64_parity"]["kernel"] = ("k_render_px64 (float64, one pixel per wave, samples summed in sample "
                                          "order): the reference's arithmetic, bit-exact against the oracle")
        obvh = dataclasses.replace(opts, flags=opts.flags | RT_FLAG_NO_BINNING)
        extra["bvh_path"] = sub_measure(ds, obvh, fb, stream, k_extra, 1, base_key + f"_flags{RT_FLAG_NO_BINNING}")
        extra["bvh_path"]["kernel"] = ("k_render_fast<false> with RT_FLAG_NO_BINNING: every camera and shadow ray "
                                       "through the BVH (wave-coherent traversal, fp32), no per-pixel or light-cell "
                                       "lists — the path of scenes outside the one-mesh / one-plane envelope")

    value = rays_frame * args.steps / elapsed / 1e6
    # SURVEY 8(d)'s per-ray BVH byte model over this launch's rays (what a
    # per-ray BVH tracer would read; these kernels skip most of it)
    bvh_model_bytes = (counters["lane_node_visits"] * 2 * SURVEY_BOX_BYTES
                       + counters["lane_tri_tests"] * SURVEY_TRI_BYTES + rows * W * PIXEL_BYTES)
    workload_key = (f"{args.config.lower()}_{W}x{H}_m{m}_world{world}" + ("_fp64" if fp64 else "")
                    + (f"_flags{args.flags}" if args.flags else ""))
    pmc = load_pmc(workload_key)
    roof = {"bound": "issue", "achieved": None, "peak": VALU_PEAK_GINST, "unit": "G wave64 VALU inst/s",
            "frac": None, "traffic": None}
    if pmc is not None:
        c = pmc["counters_mean_per_dispatch"]
        sec = render_ms * 1e-3
        roof.update(issue_roofline(c, sec))
        if kinds == 15 and not fp64:
            add_net_of_spills(roof, "k_render_mix1ILi2ELi4E")
        elif fp64:
            add_net_of_spills(roof, "k_render_px64ILi4ELi1E")
        if "hbm_bytes_per_launch" in pmc:
            roof["traffic"] = int(pmc["hbm_bytes_per_launch"])
            roof["hbm_gbs"] = round(pmc["hbm_bytes_per_launch"] / sec / 1e9, 1)
            roof["hbm_frac"] = round(pmc["hbm_bytes_per_launch"] / sec / 1e9 / HBM_PEAK_GBS, 4)
        roof["pmc"] = f"profiles/pmc_summary.json[{workload_key}] (sources {pmc['source_hash']}): {pmc.get('note', '')}"
    else:
        roof["pmc"] = "no PMC summary for these native sources (profiles/pmc_summary.json): achieved / frac null"
    roof.update({
        "kernel": "render kernels: " + kernel_desc,
        "kernel_ms": round(render_ms, 4),
        "setup_ms": round(setup_ms, 4),
        "call_ms": round(call_ms, 4),
        "definition": ("achieved = PMC SQ_INSTS_VALU of the render kernels per call / their duration (HIP events "
                       "inside the library, RT_FLAG_TIMING pass after the timed region); peak = 1024 SIMDs x "
                       f"{CLOCK_GHZ} GHz / {VALU_CYCLES} cycles per wave64 VALU instruction; salu_frac likewise "
                       "against one scalar instruction per CU per cycle; traffic = PMC HBM bytes per call "
                       "(2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md)"),
        "setup": ("per-call camera-dependent build on the device (rt_frame.hip, three launches: faces into "
                  "per-pixel list slots + skip cells; pixel records; lean / general lists), inside every timed step"),
        "survey_bvh_model_gbs": round(bvh_model_bytes / (render_ms * 1e-3) / 1e9, 1),
        "survey_bvh_model_note": ("SURVEY 8(d) bytes of a per-ray BVH tracer (32 B/box, 36 B/triangle, 12 B/pixel) "
                                  "from one instrumented BVH-only launch, over the render kernels' time: a model, "
                                  "not traffic (the kernels share each record fetch across 64 lanes)"),
        "bvh_model_lane_node_visits": counters["lane_node_visits"],
        "bvh_model_lane_tri_tests": counters["lane_tri_tests"],
    })

    if rank == 0:
        out = {
            "metric": ("Mray/s (primary+shadow) on bunny.geom 1080p/256spp; 1/2/4/8-GPU scaling"
                       if args.config == "C3" else f"Mray/s (primary+shadow) on {args.config}"),
            "value": round(value, 2),
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64" if fp64 else "f32",
            "data": {"bunny": "synthetic rays over the reference's bunny.geom fixture (69,451 triangles)",
                     "boxes2": "synthetic rays over the reference's boxes2.nim scene",
                     "torus": "synthetic rays over a deterministic procedural 1M-triangle torus",
                     "mix": "synthetic rays over a test scene of this build (mesh-mix)"}[scene_name],
            "config": {
                "workload": (f"{desc}, {W}x{H}, akGrid {m}x{m} = {m * m} spp, "
                             + ("fp64 parity mode (k_render_px64: the reference's arithmetic, bit-exact "
                                "against the oracle), " if fp64 else "fp32, ")
                             + (f"{BAND_H}-row bands round-robin over {world} ranks (one GPU each) + RCCL gather "
                                "to rank 0" if distributed else "one whole-frame call per step on one GPU")
                             + "; every step builds its camera-dependent data on the device"),
                "width": W, "height": H, "spp": m * m, "triangles": info["num_triangles"],
                "bvh_nodes": info["num_bvh_nodes"], "primary_rays_per_frame": prim_frame,
                "shadow_rays_per_frame": shadow_frame, "parallelism": f"bands{world}",
                "scene_setup_s": round(setup_s, 3), "scene_setup_ms_lib": round(info["build_ms"], 1),
                "first_frame_ms": None if first_frame_ms is None else round(first_frame_ms, 3),
                "camera_change_frame_ms": None if camera_change_ms is None else round(camera_change_ms, 3),
                "lean_pixel_groups": lean_groups, "general_pixel_groups": general_groups,
                "batched_general_groups": batched_groups, "batch_fallback_groups": batch_fallback,
                "bvh_builder": {"sah": "host binned SAH", "ploc": "device PLOC"}[args.bvh],
            },
            "roofline": roof,
            "cpu_baseline": None,
            # build provenance: the library's embedded source hash against this tree's
            "build": {"library_sources": library_source_hash(), "tree_sources": kernel_source_hash(),
                      "match": library_source_hash() == kernel_source_hash()},
        }
        if frame_check is not None:
            out["frame_check"] = frame_check
        out.update(extra)
        if world == 1 and not args.no_cpu:
            # the reference's brute-force mesh loop is infeasible past ~200k
            # triangles (~1e11 triangle tests per 4K row): same-BVH only there
            if info["num_triangles"] <= 200_000:
                out["cpu_baseline"] = cpu_baseline(scene, W, H, args.cpu_seconds)
            # the same algorithm class on the CPU (BVH), so the
            # GPU/CPU ratio is also judged against a fair CPU implementation
            out["cpu_baseline_same_bvh"] = cpu_baseline(scene, W, H, args.cpu_seconds, bvh=True)
        print(json.dumps(out), file=json_out, flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
