"""GPU output pass: rt_ppm_encode_device (writePpm's quantisation,
framebuf.nim:55-93) byte-exact against the host quantiser, which
test_abi.py pins to the oracle."""
import numpy as np
import pytest

from rtmi import Antialias, Options, Precision, akGrid, scenes
from rtmi.framebuf import to_uint

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("bits,srgb", [(8, True), (8, False), (16, True), (16, False), (5, True)])
@pytest.mark.parametrize("w,h", [(64, 48), (7, 3)])   # 7x3: component count not a multiple of 4
def test_ppm_encode_exact(gpu, bits, srgb, w, h):
    import torch

    from rtmi.renderer import ppm_encode_device
    rng = np.random.default_rng(bits * 10 + w)
    data = (rng.random((h, w, 3)) * 1.3 - 0.15).astype(np.float32)
    data.reshape(-1)[:5] = [0.0031308, 0.5 / 255, np.nan, -0.0, 1.0]
    d = torch.from_numpy(data.reshape(-1)).cuda()
    header, payload = ppm_encode_device(d, w, h, bits, srgb)
    got = payload.cpu().numpy()
    q = to_uint(data, bits, srgb).reshape(-1)
    want = q.astype(">u2").view(np.uint8) if bits > 8 else q
    assert header == f"P6 {w} {h} {2 ** bits - 1} ".encode()
    assert np.array_equal(got, want)


@pytest.mark.parametrize("w,h", [(64, 48), (7, 3), (1, 1)])
def test_rgba_encode_exact(gpu, w, h):
    """ImageRGBA.copyFrom on the GPU (rt_rgba_encode_device) byte-exact
    against the host mirror, which test_abi.py pins to the oracle."""
    import torch

    from rtmi.framebuf import to_rgba
    from rtmi.renderer import rgba_encode_device
    rng = np.random.default_rng(w * 7 + h)
    data = (rng.random((h, w, 3)) * 1.6 - 0.3).astype(np.float32)
    flat = data.reshape(-1)
    specials = np.array([0.5 / 255, 254.5 / 255, 1.0, np.nan, np.inf, -1e30, 2.0, -0.0, 1e7], np.float32)
    flat[:min(len(specials), flat.size)] = specials[:flat.size]
    out = rgba_encode_device(torch.from_numpy(flat).cuda(), w, h, alpha=0xC8)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), to_rgba(data, 0xC8))


def test_write_ppm_device_matches_host_writer(gpu, tmp_path):
    import torch

    from rtmi.framebuf import writePpm
    from rtmi.renderer import DeviceScene, write_ppm_device
    ds = DeviceScene(scenes.mesh_bunny())
    opts = Options(width=160, height=96, antialias=Antialias(akGrid, 2), bias=1e-4, precision=Precision.fp32)
    fb = torch.zeros(160 * 96 * 3, dtype=torch.float32, device="cuda")
    ds.render_device(opts, fb)
    a, b = tmp_path / "gpu.ppm", tmp_path / "host.ppm"
    assert write_ppm_device(fb, 160, 96, str(a), 16, True)
    assert writePpm(fb.cpu().numpy().reshape(96, 160, 3), str(b), 16, True)
    assert a.read_bytes() == b.read_bytes()
