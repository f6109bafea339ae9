"""N-GPU projection of a BASELINE config's band-sharded frame, simulated on one GPU.

    CONFIG=C3|C4|C5 REPS=5 BANDS=4[,16,...] WORLDS=1,2,4,8 python tools/scaling_sim.py

For N in 1, 2, 4, 8 every rank's rt_render_bands_device call is timed (HIP
events, median of REPS: `world{N}_max_ms`, the slowest rank) and called REPS
times back to back with no host sync (`world{N}_b2b_max_ms`: a rank's step
loop, where a call's per-call build overlaps the previous call's render —
rt_scene bstream). On top of the slowest rank, bench.py's N-GPU step also
runs on rank 0: the on-GPU un-interleave of the gathered bands
(`unshard_ms`, measured here for the N-rank layout) and the RCCL gather,
which overlaps the next frame's render (bench.py gathers frame k while
frame k+1 renders) and so only shows when it takes longer than a render:
`gather_model_ms` = the bytes rank 0 receives / (N - 1 xGMI links x
LINK_GBS, default 50 GB/s per link and direction — a conservative figure
for MI355X's ~153 GB/s links). The projection:
    step_N = b2b_max_N + unshard_N + max(0, gather_N - b2b_max_N)
and `projected_speedup_N` = step_1 / step_N (`projected_speedup_loop_N`: with
rank 0's measured loop — band call + un-interleave back to back — in place of
adding the un-interleave to the slowest rank), step_1 = the faster of the
whole-frame call and the one-rank band call, both back to back (the
one-GPU bench line runs the whole frame).
Prints one JSON line per band height.
"""
import json
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "nim-raytracer_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from bench import CONFIGS, _scene  # noqa: E402
from rtmi import Antialias, Options, Precision, akGrid  # noqa: E402
from rtmi.dist import band_rows  # noqa: E402
from rtmi.renderer import DeviceScene, unshard_bands_device  # noqa: E402

CFG = os.environ.get("CONFIG", "C3")
name, W, H, M, _desc = CONFIGS[CFG]
M = int(os.environ.get("GRID", M))  # akGrid m override (spp = m*m): item-length experiments
REPS = int(os.environ.get("REPS", "5"))
LINK_GBS = float(os.environ.get("LINK_GBS", "50"))
ds = DeviceScene(_scene(name))
opts = Options(width=W, height=H, antialias=Antialias(akGrid, M), bias=1e-4, precision=Precision.fp32,
               flags=int(os.environ.get("RTMI_FLAGS", "0"), 0))
stream = torch.cuda.current_stream()


def timed(fn, reps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(reps):
        fn()
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


# RSTREAMS=2 (A/B): a rank's pipelined back-to-back calls alternate two
# streams and two band buffers (measured with a library build that let call
# k+1 render into call k's tail: slower); 1: one
# stream, the projection's measurement
RSTREAMS = int(os.environ.get("RSTREAMS", "1"))
stream2 = torch.cuda.Stream()


def timed_two(fn, reps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    stream2.wait_stream(stream)
    for k in range(reps):
        fn(k, stream if k % 2 == 0 else stream2)
    stream.wait_stream(stream2)
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
for band_h in [int(b) for b in os.environ.get("BANDS", "4").split(",")]:
    res = {"config": CFG, "width": W, "height": H, "spp": M * M, "band_h": band_h, "reps": REPS, "rstreams": RSTREAMS,
           "link_gbs_model": LINK_GBS}
    ds.render_device(opts, fb, stream=stream, stats=False)
    res["whole_frame_b2b_ms"] = round(timed(lambda: ds.render_device(opts, fb, stream=stream, stats=False), REPS), 4)
    for world in [int(w) for w in os.environ.get("WORLDS", "1,2,4,8").split(",")]:
        rows = band_rows(H, band_h, world)
        buf = torch.zeros(rows * W * 3, dtype=torch.float32, device="cuda")
        bufs2 = [buf, torch.zeros_like(buf)]
        order = list(range(world))
        if os.environ.get("RANK_ORDER") == "reverse":  # measurement-order check
            order.reverse()
        per, b2b = [0.0] * world, [0.0] * world
        for rank in order:
            ts = []
            for k in range(2):  # warm: the first launch of a mapping measures its launch order
                ds.render_bands_device(opts, buf, band_h, rank, world, stream=stream2 if RSTREAMS == 2 and k else stream,
                                       stats=False)
            torch.cuda.synchronize()
            for _ in range(REPS):
                ts.append(timed(lambda: ds.render_bands_device(opts, buf, band_h, rank, world, stream=stream,
                                                               stats=False), 1))
            per[rank] = sorted(ts)[len(ts) // 2]
            if RSTREAMS == 2 and ds.last_pipelined():
                b2b[rank] = timed_two(lambda k, st: ds.render_bands_device(opts, bufs2[k % 2], band_h, rank, world,
                                                                           stream=st, stats=False), REPS)
            else:
                b2b[rank] = timed(lambda: ds.render_bands_device(opts, buf, band_h, rank, world, stream=stream,
                                                                 stats=False), REPS)
            if rank == 0:
                res[f"world{world}_split"] = list(ds.last_split())
        gathered = torch.zeros(world * rows * W * 3, dtype=torch.float32, device="cuda")
        unshard = timed(lambda: unshard_bands_device(gathered, fb, W, H, band_h, world, stream=stream), REPS)
        recv_bytes = (world - 1) * rows * W * 12
        gather = recv_bytes / (max(1, world - 1) * LINK_GBS * 1e9) * 1e3 if world > 1 else 0.0
        b2b_max = max(b2b)
        step = b2b_max + (unshard if world > 1 else 0.0) + max(0.0, gather - b2b_max)
        if world > 1:
            # rank 0's own loop as bench.py runs it: its band call, then the
            # un-interleave of the previous frame on the same stream (which
            # can fill the gap while the next call's build finishes), back to
            # back; the RCCL gather's own kernels on rank 0 are not modelled
            def rank0_step():
                ds.render_bands_device(opts, buf, band_h, 0, world, stream=stream, stats=False)
                unshard_bands_device(gathered, fb, W, H, band_h, world, stream=stream)
            r0 = timed(rank0_step, REPS)
            step_loop = max([r0] + b2b[1:]) + max(0.0, gather - b2b_max)
            res[f"world{world}_rank0_loop_ms"] = round(r0, 4)
            res[f"world{world}_step_loop_ms"] = round(step_loop, 4)
        res[f"world{world}_ranks_ms"] = [round(x, 4) for x in per]
        res[f"world{world}_ranks_b2b_ms"] = [round(x, 4) for x in b2b]
        res[f"world{world}_max_ms"] = round(max(per), 4)
        res[f"world{world}_mean_ms"] = round(sum(per) / world, 4)
        res[f"world{world}_b2b_max_ms"] = round(b2b_max, 4)
        res[f"world{world}_unshard_ms"] = round(unshard, 4)
        res[f"world{world}_gather_model_ms"] = round(gather, 4)
        res[f"world{world}_step_ms"] = round(step, 4)
    step1 = min(res["whole_frame_b2b_ms"], res.get("world1_b2b_max_ms", res["whole_frame_b2b_ms"]))
    res["step1_ms"] = step1
    for w in (2, 4, 8):
        if f"world{w}_step_ms" in res:
            res[f"projected_speedup_{w}"] = round(step1 / res[f"world{w}_step_ms"], 2)
        if f"world{w}_step_loop_ms" in res:
            res[f"projected_speedup_loop_{w}"] = round(step1 / res[f"world{w}_step_loop_ms"], 2)
    if "world8_max_ms" in res and "world1_max_ms" in res:
        res["render_speedup_8"] = round(res["world1_max_ms"] / res["world8_max_ms"], 2)
        res["b2b_speedup_8"] = round(res["world1_b2b_max_ms"] / res["world8_b2b_max_ms"], 2)
    print(json.dumps(res), flush=True)
