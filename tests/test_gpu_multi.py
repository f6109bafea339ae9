"""One-process multi-GPU frames (rt_multi_*, csrc/rt_multi.cpp; SURVEY.md
8(b) rt_render_frame_multi). On a one-GPU box the device list repeats
device 0, which runs the whole band layout, per-rank scenes, copies into
devices[0] and un-interleave; frames and Stats must equal the single-scene
frame bit for bit."""
import numpy as np
import pytest

from rtmi import Antialias, Options, Precision, akGrid, scenes
from rtmi.renderer import DeviceScene, MultiDeviceScene

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world,band_h", [(1, 4), (3, 4), (4, 7), (8, 16)])
@pytest.mark.parametrize("prec", [Precision.fp32, Precision.fp64])
def test_multi_frame_equals_single(gpu, world, band_h, prec):
    import torch
    scene = scenes.mesh_mix()
    w, h = 150, 97
    opts = Options(width=w, height=h, antialias=Antialias(akGrid, 2), bias=1e-4, precision=prec)
    ref = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    sref = DeviceScene(scene).render_device(opts, ref)
    ms = MultiDeviceScene(scene, devices=[0] * world, band_h=band_h)
    out = torch.zeros_like(ref)
    for _ in range(2):  # second frame: the ranks' longest-first launch orders
        out.zero_()
        assert ms.render_frame_device(opts, out) == sref
        assert torch.equal(out, ref)
    fb = np.zeros((h, w, 3), np.float32)
    assert ms.render_frame(opts, fb) == sref
    assert np.array_equal(fb, ref.view(h, w, 3).cpu().numpy())
    ms.close()


def test_multi_rejects_bad_devices(gpu):
    from rtmi._lib import RtmiError
    with pytest.raises(RtmiError):
        MultiDeviceScene(scenes.spheres_warm(3), devices=[0, 99])
