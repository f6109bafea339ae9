#!/usr/bin/env python3
"""Benchmark: Mray/s (primary + shadow) on bunny.geom, 1920x1080, 256 spp.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

One step = one full frame of BASELINE config C3 (mesh-bunny layout: baked
bunny.geom 69,451 triangles + ground plane, 2 distant lights, akGrid 16x16 =
256 samples per pixel, fp32 performance mode) rendered from a scene resident
in HBM into a device framebuffer. With N GPUs the SAME frame is cut into
4-row bands dealt round-robin to the ranks, each rank renders its bands and
one RCCL gather + an on-GPU un-interleave assembles the frame on rank 0
(strong scaling; every gather is inside the timed region, frame k's
overlapping frame k+1's render from a second band buffer).

Printed (rank 0, one JSON line): value = (primary + shadow rays of all ranks)
x K / max-over-ranks wall time, plus
  roofline     — the render call (C3-C5, one mesh on one ground plane: the
                 merged kernel k_render_mix1 — general pixels, then lean
                 pixels; elsewhere the two-class launch k_render_gen +
                 k_render_lean, or k_render_fast), HIP events on the stream it
                 runs on, against the 8 TB/s HBM peak.
                 `achieved` = SURVEY 8(d)'s algorithmic bytes per ray — 32 B
                 per BVH box and 36 B per triangle the ray is tested against,
                 + 12 B per pixel — summed over the rays with the per-lane
                 counts of the algorithm the kernels execute (binned face
                 lists, pixel records, BVH only for left-over lanes; from one
                 instrumented launch), / the call's duration. `traffic` = the
                 PMC-measured HBM bytes per launch (profiles/, or null); the
                 kernels are not HBM-bound (one scalar record fetch serves 64
                 lanes, the working set lives in the caches): `issue` holds
                 the VALU / SALU issue utilisation from the committed PMC
                 instruction counts, the actual limiter. The per-ray BVH model
                 of round 1 (every ray traverses the scene BVH) is kept as
                 `survey_bvh_model_gbs` for comparison only;
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
NODE_BYTES = 64        # what the kernel fetches: one BvhNode record (two child boxes + refs)
TRI_BYTES = 64         # one TriFast record (v0, e2, -e1, -n, face id)
BAND_H = 4             # rows per band (round-robin over ranks)


def _scene(name):
    from rtmi import scenes
    return {"bunny": scenes.mesh_bunny, "boxes2": scenes.boxes2, "torus": scenes.torus_scene}[name]()


# BASELINE.json configs on one GPU (C4/C5 are quoted on 8 GPUs; at N=1 this is
# one GPU's whole frame, at N>1 the band-sharded frame)
CONFIGS = {
    "C2": ("boxes2", 1920, 1080, 8, "C2: boxes2.nim (16 analytic primitives, 1 distant light)"),
    "C3": ("bunny", 1920, 1080, 16, "C3: bunny.geom baked x30 + ground plane, mesh-bunny.nim lights/camera"),
    "C4": ("bunny", 3840, 2160, 32, "C4: bunny.geom baked x30 + ground plane, mesh-bunny.nim lights/camera"),
    "C5": ("torus", 3840, 2160, 64, "C5: 1,000,000-triangle procedural torus + ground, mesh-bunny.nim lights/camera"),
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
    ap.add_argument("--bvh", default="sah", choices=["sah", "ploc"],
                    help="mesh BVH builder: host binned SAH (default) or device PLOC")
    ap.add_argument("--flags", type=int, default=0, help="rt_options.flags (1 = any-hit shadows)")
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
CLOCK_GHZ = 2.4        # peak engine clock
VALU_CYCLES = 2        # a wave64 fp32 VALU instruction per SIMD (tools/micro/issue_rate.hip)


def load_pmc(workload_key):
    """Per-launch PMC figures of the render call from the committed summary
    (profiles/pmc_summary.json, tools/pmc_summary.py), or None."""
    p = os.path.join(REPO, "profiles", "pmc_summary.json")
    try:
        with open(p) as f:
            return json.load(f).get(workload_key)
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from rtmi import Antialias, Options, Precision, akGrid, scenes
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
    opts = Options(width=W, height=H, antialias=Antialias(akGrid, m), bias=1e-4,
                   precision=Precision.fp32, flags=args.flags)
    stream = torch.cuda.current_stream()
    # the first frame of this camera and image size also builds its
    # camera-dependent bins (pixel face lists, pixel records, lean/general
    # lists): timed on its own, reported beside the steady-state frame
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
        # un-interleave into the frame buffer, in stream order
        if pending[0] is not None:
            pending[0].wait()
            pending[0] = None
            if rank == 0:
                unshard_bands_device(gathered, fb, W, H, BAND_H, world, stream=stream)

    def step(time_kernel=None):
        # render this rank's bands (world == 1: the whole frame, one band set)
        buf = local_bufs[nframe[0] % 2]
        nframe[0] += 1
        if time_kernel is not None:
            time_kernel[0].record(stream)
        if distributed:
            ds.render_bands_device(opts, buf, BAND_H, rank, world, stream=stream, stats=False)
        else:
            ds.render_device(opts, fb, stream=stream, stats=False)
        if time_kernel is not None:
            time_kernel[1].record(stream)
        if distributed:
            finish_frame()  # frame k-1, whose gather overlapped this render
            pending[0] = gather_bands(buf, gathered if rank == 0 else None, rows * W * 3, async_op=True)

    # warmup (+ the deterministic per-frame ray counts)
    # two instrumented launches (RT_FLAG_COUNT_TRAVERSAL): the per-ray BVH
    # visit / test counts of SURVEY 8(d)'s algorithmic bytes (BVH for every
    # ray: RT_FLAG_NO_BINNING), and the records the kernel really fetches
    # (camera / shadow rays searching their pixel lists and light grids)
    from rtmi.abi import RT_FLAG_COUNT_TRAVERSAL, RT_FLAG_NO_BINNING
    import dataclasses
    copts = dataclasses.replace(opts, flags=opts.flags | RT_FLAG_COUNT_TRAVERSAL | RT_FLAG_NO_BINNING)
    st = ds.render_bands_device(copts, local_buf, BAND_H, rank, world, stream=stream, stats=True)
    counters = ds.last_counters()
    kopts = dataclasses.replace(opts, flags=opts.flags | RT_FLAG_COUNT_TRAVERSAL)
    ds.render_bands_device(kopts, local_buf, BAND_H, rank, world, stream=stream, stats=False)
    kcounters = ds.last_counters()
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
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    finish_frame()  # the last frame's gather + un-interleave, inside the timed region
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if distributed:
        e = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / max(1, args.steps)
    lean_groups, general_groups = ds.last_split()
    kinds = ds.last_lean_kernel()
    lean_k = {0: None, 1: "k_render_lean", 2: "k_render_lean1q (one-plane lean pixels)", 3: None}[kinds & 3]
    gen_k = {0: "k_render_fast<false>", 1: "k_render_gen", 2: "k_render_gen1 (one-plane general pixels)",
             3: None}[kinds >> 2 & 3]
    kernel_desc = ("k_render_mix1 (one-plane scene: general pixels, then lean pixels, one merged kernel)"
                   if kinds == 15 else f"{gen_k} + {lean_k} (two-class launch)" if lean_k else gen_k)
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

    value = rays_frame * args.steps / elapsed / 1e6
    # algorithmic bytes of one launch on this rank, SURVEY.md 8(d): per ray
    # 32 B x boxes tested + 36 B x triangles tested + 12/spp B, summed over
    # the launch's rays with the per-lane counts of the executed algorithm
    # (binned lists, pixel records, BVH for left-over lanes only)
    bytes_launch = (kcounters["lane_node_visits"] * 2 * SURVEY_BOX_BYTES
                    + kcounters["lane_tri_tests"] * SURVEY_TRI_BYTES + rows * W * PIXEL_BYTES)
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    # round 1's model: every ray traverses the scene BVH (what a per-ray
    # BVH tracer would need; the kernels skip most of it)
    bvh_model_bytes = (counters["lane_node_visits"] * 2 * SURVEY_BOX_BYTES
                       + counters["lane_tri_tests"] * SURVEY_TRI_BYTES + rows * W * PIXEL_BYTES)
    # what the wave-coherent kernels request: one record fetch serves all 64
    # lanes of a wave (binned searches: + a 4-B list entry per face)
    fetch_bytes = (kcounters["wave_node_fetches"] * NODE_BYTES + kcounters["wave_tri_fetches"] * (TRI_BYTES + 4)
                   + rows * W * PIXEL_BYTES)
    workload_key = f"{args.config.lower()}_{W}x{H}_m{m}_world{world}"
    pmc = load_pmc(workload_key)
    traffic = None if pmc is None or "hbm_bytes_per_launch" not in pmc else float(pmc["hbm_bytes_per_launch"])
    issue = None
    if pmc is not None and "SQ_INSTS_VALU" in pmc.get("counters_mean_per_dispatch", {}):
        c = pmc["counters_mean_per_dispatch"]
        cyc = kern_ms * 1e-3 * CLOCK_GHZ * 1e9
        issue = {"valu_busy": round(c["SQ_INSTS_VALU"] * VALU_CYCLES / SIMDS / cyc, 3),
                 "salu_busy": round(c["SQ_INSTS_SALU"] / (SIMDS // 4) / cyc, 3),
                 "note": ("PMC instruction counts per call (committed summary) over this run's call time at "
                          f"{CLOCK_GHZ} GHz: VALU {VALU_CYCLES} cycles per wave64 instruction per SIMD, SALU one "
                          "instruction per cycle per CU (shared by its 4 SIMDs)")}

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
            "dtype": "f32",
            "data": {"bunny": "synthetic rays over the reference's bunny.geom fixture (69,451 triangles)",
                     "boxes2": "synthetic rays over the reference's boxes2.nim scene",
                     "torus": "synthetic rays over a deterministic procedural 1M-triangle torus"}[scene_name],
            "config": {
                "workload": (f"{desc}, {W}x{H}, akGrid {m}x{m} = {m * m} spp, fp32, {BAND_H}-row bands "
                             f"round-robin over {world} GPU(s) + RCCL gather to rank 0"),
                "width": W, "height": H, "spp": m * m, "triangles": info["num_triangles"],
                "bvh_nodes": info["num_bvh_nodes"], "primary_rays_per_frame": prim_frame,
                "shadow_rays_per_frame": shadow_frame, "parallelism": f"bands{world}",
                "scene_setup_s": round(setup_s, 3), "scene_setup_ms_lib": round(info["build_ms"], 1),
                "first_frame_ms": None if first_frame_ms is None else round(first_frame_ms, 1),
                "lean_pixel_groups": lean_groups, "general_pixel_groups": general_groups,
                "batched_general_groups": batched_groups, "batch_fallback_groups": batch_fallback,
                "bvh_builder": {"sah": "host binned SAH", "ploc": "device PLOC"}[args.bvh],
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": "render call: " + kernel_desc,
                "kernel_ms": round(kern_ms, 4),
                "bytes_per_launch": int(bytes_launch),
                "definition": ("SURVEY 8(d) per-ray bytes (32 B/BVH box + 36 B/triangle tested, 12 B/pixel) over "
                               "the per-lane tests the kernels execute (binned face lists, pixel records, BVH for "
                               "left-over lanes)"),
                "limiter": ("instruction issue (SALU + VALU), not HBM: one scalar record fetch serves 64 lanes and "
                            "the records live in the caches (traffic << achieved)"),
                "issue": issue,
                "record_fetch_bytes_per_launch": int(fetch_bytes),
                "record_fetch_gbs": round(fetch_bytes / (kern_ms * 1e-3) / 1e9, 1),
                "survey_bvh_model_gbs": round(bvh_model_bytes / (kern_ms * 1e-3) / 1e9, 1),
                "kernel_lane_node_visits": kcounters["lane_node_visits"],
                "kernel_lane_tri_tests": kcounters["lane_tri_tests"],
                "kernel_wave_node_fetches": kcounters["wave_node_fetches"],
                "kernel_wave_tri_fetches": kcounters["wave_tri_fetches"],
                "bvh_model_lane_node_visits": counters["lane_node_visits"],
                "bvh_model_lane_tri_tests": counters["lane_tri_tests"],
            },
            "cpu_baseline": None,
        }
        if frame_check is not None:
            out["frame_check"] = frame_check
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
