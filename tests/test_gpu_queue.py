"""Render queue (rt_queue_*, rtmi.renderer.RenderQueue): the WorkerPool that
raytracer.nim and gui.nim drive (src/concurrency/workerpool.nim,
src/raytracer.nim:13-38, src/gui.nim:206-280), over the GPU. Frames and
summed Stats must equal direct rt_render_lines calls of the same lines."""
import time

import numpy as np
import pytest

from rtmi import Antialias, Options, Precision, akGrid, akNone, scenes
from rtmi._lib import RtmiError
from rtmi.abi import RT_QUEUE_RUNNING, RT_QUEUE_SHUTDOWN, RT_QUEUE_STOPPED
from rtmi.renderer import DeviceScene, initRenderWorkers
from rtmi.scene import Stats

pytestmark = pytest.mark.gpu


def _drain(q, n, timeout=60.0):
    got, total = [], Stats()
    t0 = time.time()
    while len(got) < n:
        ok, r = q.tryRecvResult()
        if ok:
            got.append(r.line)
            total += r.stats
        elif time.time() - t0 > timeout:
            raise TimeoutError(f"{len(got)} of {n} responses")
        else:
            time.sleep(0.0005)
    return got, total


@pytest.mark.parametrize("prec", [Precision.fp32, Precision.fp64])
def test_gui_progressive_levels_match_direct(gpu, prec):
    """gui.nim's loop: maxStep 4, levels step 4, 2, 1, each queueing
    countup(0, h-1, step) with (step, maxStep) and receiving every response."""
    scene = scenes.mesh_mix()
    w, h, max_step = 96, 70, 4
    opts = Options(width=w, height=h, antialias=Antialias(akGrid, 2), bias=1e-4, precision=prec)
    ds = DeviceScene(scene)
    q = initRenderWorkers(ds, numActiveWorkers=6, poolSize=8)
    q.waitForReady()
    assert q.state() == RT_QUEUE_STOPPED and q.isReady()
    assert q.start() and q.state() == RT_QUEUE_RUNNING
    fb = np.zeros((h, w, 3), np.float32)
    ref = np.zeros_like(fb)
    step = max_step
    while step >= 1:
        lines = list(range(0, h, step))
        for y in lines:
            q.queueWork(opts, fb, y, step, max_step)
        got, total = _drain(q, len(lines))
        assert got == lines  # one response per message, in queue order
        want = ds.render_lines(opts, ref, 0, h, step, max_step)
        assert total == want, step
        assert np.array_equal(fb, ref), step
        step //= 2
    assert q.stop() and q.state() == RT_QUEUE_STOPPED
    assert q.shutdown() and q.state() == RT_QUEUE_SHUTDOWN
    assert q.close()


def test_raytracer_main_flow_and_commands(gpu):
    """raytracer.nim:main: start, queue every line with step 0 (= 1), sum the
    responses; plus workerpool.nim's command rules: start only when stopped,
    stop only when running, work queued while stopped waits, reset drops
    queued work, nothing is accepted after shutdown, close needs shutdown."""
    scene = scenes.spheres_warm(3)
    w, h = 64, 48
    opts = Options(width=w, height=h, antialias=Antialias(akNone, 1), bias=1e-4, precision=Precision.fp32)
    ds = DeviceScene(scene)
    q = initRenderWorkers(ds)
    fb = np.zeros((h, w, 3), np.float32)
    assert not q.stop()             # not running
    for y in range(h):              # queued while stopped: nothing happens
        q.queueWork(opts, fb, y)
    time.sleep(0.05)
    assert q.tryRecvResult() == (False, None)
    assert q.start() and not q.start()
    got, total = _drain(q, h)
    assert sorted(got) == list(range(h))
    ref = np.zeros_like(fb)
    assert total == ds.render_lines(opts, ref, 0, h)
    assert np.array_equal(fb, ref)
    # reset drops queued work and undelivered responses, leaves the queue stopped
    assert q.stop()
    for y in range(h):
        q.queueWork(opts, fb, y)
    assert q.reset() and q.state() == RT_QUEUE_STOPPED
    assert q.start()
    time.sleep(0.05)
    assert q.tryRecvResult() == (False, None)
    assert not q.close()            # close needs shutdown
    assert q.shutdown() and not q.shutdown()
    with pytest.raises(RtmiError):
        q.queueWork(opts, fb, 0)
    assert q.close()


def test_failed_line_reports_its_error(gpu):
    ds = DeviceScene(scenes.spheres_warm(3))
    q = initRenderWorkers(ds)
    bad = Options(width=32, height=8, antialias=Antialias(akGrid, 0), bias=1e-4, precision=Precision.fp32)
    fb = np.zeros((8, 32, 3), np.float32)
    q.queueWork(bad, fb, 0)
    q.start()
    t0 = time.time()
    while True:
        try:
            ok, _ = q.tryRecvResult()
        except RtmiError as e:
            assert "grid_size" in str(e)
            break
        assert time.time() - t0 < 30
        time.sleep(0.001)
    q.shutdown()
    q.close()


def test_queue_progressive_frame_matches_oracle(gpu, oracle_mod):
    """The queue-driven gui.nim loop against the oracle itself (not only against
    direct calls): float64 parity mode, maxStep 4 -> 2 -> 1 over every
    countup(0, h-1, step) line, the oracle's renderLine (renderer.nim:162-211)
    called for the same lines in the same order — frames bit-identical after
    every level, Stats equal in total."""
    scene = scenes.mesh_mix()
    w, h, max_step = 80, 56, 4
    opts = Options(width=w, height=h, antialias=Antialias(akGrid, 2), bias=1e-4, maxRayDepth=5,
                   precision=Precision.fp64)
    ds = DeviceScene(scene)
    q = initRenderWorkers(ds, numActiveWorkers=4, poolSize=8)
    q.waitForReady()
    assert q.start()
    o = oracle_mod.OracleScene(scene)
    fb = np.zeros((h, w, 3), np.float32)
    ref = np.zeros_like(fb)
    tot_g, tot_r = Stats(), Stats()
    step = max_step
    while step >= 1:
        lines = list(range(0, h, step))
        for y in lines:
            q.queueWork(opts, fb, y, step, max_step)
        _, st = _drain(q, len(lines))
        tot_g += st
        for y in lines:
            tot_r += o.render_line(opts, ref, y, step, max_step)
        assert np.array_equal(fb, ref), step
        step //= 2
    assert tot_g == tot_r
    assert q.stop() and q.shutdown() and q.close()
