"""Two-class launches of the float32 kernel (rtmi.cpp split_lists): lean
pixels — no camera ray can hit the mesh, every light is a distant light whose
shadow rays provably miss it — render in k_render_lean from a per-launch
list (k_render_lean1 in one-plane scenes, RT_FLAG_NO_LEAN1 turns it off), the rest in
k_render_gen1 (one-plane scenes, RT_FLAG_NO_GEN1), k_render_gen (several samples per lane through each face
list; a pixel whose shadow rays need the BVH falls back to the one-sample
loop) or, where that does not apply, k_render_fast. Scheduling only: frames
and Stats must be bit-identical to the general pixels in k_render_fast
(RT_FLAG_NO_BATCH), to the one-kernel launch (RT_FLAG_NO_SPLIT) and to the
BVH-only kernel (RT_FLAG_NO_BINNING: no pixel records, no lean path at all),
whose parity with the oracle test_gpu_parity.py pins.

Also the cases the round-1 review found uncovered: shadow skip bits in a
kernel compiled with reflection (they may apply at the camera level only),
stochastic samplers and progressive passes (step > 1) against the records."""
import pytest

from rtmi import Antialias, Options, Precision, akGrid, scenes
from rtmi.abi import (RT_FLAG_BATCH_FALLBACK, RT_FLAG_NO_BATCH, RT_FLAG_NO_BINNING, RT_FLAG_NO_GEN1,
                      RT_FLAG_NO_LEAN1, RT_FLAG_NO_MIX, RT_FLAG_NO_REORDER, RT_FLAG_NO_SPLIT)
from rtmi.dist import band_rows
from rtmi.glm import X_AXIS, degToRad, inverse, mat4, rotate, translate, vec3
from rtmi.renderer import DeviceScene
from rtmi.scene import akCorrelatedMultiJittered, akJittered, akMultiJittered

pytestmark = pytest.mark.gpu

FLAG_SETS = (0, RT_FLAG_NO_MIX, RT_FLAG_NO_LEAN1, RT_FLAG_NO_GEN1, RT_FLAG_NO_BATCH, RT_FLAG_BATCH_FALLBACK, RT_FLAG_NO_SPLIT, RT_FLAG_NO_BINNING)


def _opts(w, h, m, flags=0, aa=akGrid, bias=1e-4, seed=0):
    # NO_REORDER: a short launch (these small frames) otherwise hands its
    # groups out longest-first from a measuring launch, and such launches
    # keep the one kernel (rtmi.cpp split_lists) — the split would go untested
    return Options(width=w, height=h, antialias=Antialias(aa, m), bias=bias, precision=Precision.fp32,
                   flags=flags | RT_FLAG_NO_REORDER, seed=seed)


def _frames(ds, make_opts, y0=0, y1=None, step=1, max_step=1):
    import torch
    out = []
    for flags in FLAG_SETS:
        o = make_opts(flags)
        fb = torch.full((o.height * o.width * 3,), -7.0, dtype=torch.float32, device="cuda")
        st = ds.render_device(o, fb, y0=y0, y1=o.height if y1 is None else y1, step=step, maxStep=max_step)
        out.append((fb, st))
    return out


def _assert_same(frames, what):
    import torch
    (fa, sa) = frames[0]
    for (fb, sb), flags in zip(frames[1:], FLAG_SETS[1:]):
        assert sa == sb, (what, flags, sa, sb)
        assert torch.equal(fa, fb), (what, flags, float((fa - fb).abs().max()))


def _reflective_ground(wall):
    """The bunny over a reflective ground plane (and optionally a reflective
    back wall): pixel records exist (one mesh + planes), the kernel is
    compiled with reflection, so skip bits must only drop the mesh from the
    camera level's shadow rays, never from a reflected ray's."""
    from rtmi.scene import Material, Object, Scene, initPlane
    mesh = scenes.baked_bunny()
    mesh.objectToWorld = translate(mat4(1.0), vec3(0.0, 0.0001, -12.0))
    mesh.worldToObject = inverse(mesh.objectToWorld)
    objects = [Object("bunny", mesh, Material(albedo=vec3(0.6, 0.9, 0.2))),
               Object("ground", initPlane(objectToWorld=mat4(1.0)), Material(albedo=vec3(0.4), reflection=0.5))]
    if wall:
        w = rotate(translate(mat4(1.0), vec3(0.0, 0.0, -20.0)), X_AXIS, degToRad(90.0))
        objects.append(Object("wall", initPlane(objectToWorld=w),
                              Material(albedo=vec3(0.3, 0.3, 0.5), reflection=0.7)))
    return Scene(objects=objects, lights=scenes._warm_lights(), fov=50.0,
                 cameraToWorld=scenes._std_camera(0.0, 5.5, 1.5), bgColor=vec3(0.01, 0.03, 0.05))


SCENES = {
    "bunny": scenes.mesh_bunny,
    "torus": lambda: scenes._mesh_scene(scenes.torus_mesh(96, 48), "t", (0.9, 0.5, 0.2)),
    "mesh_mix": scenes.mesh_mix,         # point light: no lean pixels
    "two_meshes": scenes.two_meshes,     # no pixel records
}


@pytest.mark.parametrize("name", list(SCENES))
@pytest.mark.parametrize("m", [8, 10, 12, 16, 32])
def test_split_matches_one_kernel(gpu, name, m):
    """spp 64 .. 1024 incl. iteration counts that are not a multiple of the
    lean batch (m = 10: 2 iterations, m = 12: 3)."""
    ds = DeviceScene(SCENES[name]())
    _assert_same(_frames(ds, lambda f: _opts(200, 120, m, f)), (name, m))


@pytest.mark.parametrize("aa", [akJittered, akMultiJittered, akCorrelatedMultiJittered])
@pytest.mark.parametrize("m", [8, 16])
def test_split_stochastic_samplers(gpu, aa, m):
    """Jittered / (correlated) multi-jittered samples stay inside their pixel
    square, so the pixel records hold for them: same frames with and
    without records and lean kernel."""
    ds = DeviceScene(scenes.mesh_bunny())
    _assert_same(_frames(ds, lambda f: _opts(160, 96, m, f, aa=aa, seed=0x5EED)), (aa, m))


def test_split_progressive_and_row_ranges(gpu):
    """renderLine's progressive passes (step > 1: skipped pixels, block
    fills) and partial row ranges use their own per-launch lists."""
    ds = DeviceScene(scenes.mesh_bunny())
    for step, mx in ((4, 4), (2, 4), (1, 2)):
        _assert_same(_frames(ds, lambda f: _opts(192, 108, 16, f), step=step, max_step=mx), (step, mx))
    _assert_same(_frames(ds, lambda f: _opts(192, 108, 16, f), y0=37, y1=90), "rows 37..90")


def test_split_bands(gpu):
    """Multi-GPU band launches: each rank's list covers exactly its bands."""
    import torch
    ds = DeviceScene(scenes.mesh_bunny())
    w, h, world = 256, 144, 3
    rows = band_rows(h, 4, world)
    for r in range(world):
        res = []
        for flags in FLAG_SETS:
            b = torch.full((rows * w * 3,), -7.0, dtype=torch.float32, device="cuda")
            st = ds.render_bands_device(_opts(w, h, 16, flags), b, 4, r, world)
            res.append((b, st))
        _assert_same(res, ("rank", r))


@pytest.mark.parametrize("wall", [False, True])
def test_skip_bits_with_reflection(gpu, wall):
    """Reflective ground (and wall) under the bunny: the skip bits of the
    camera level must not leak into reflected rays' shadow traces."""
    ds = DeviceScene(_reflective_ground(wall))
    for m in (8, 16):
        _assert_same(_frames(ds, lambda f: _opts(240, 135, m, f)), (wall, m))


def test_split_full_c3(gpu):
    """BASELINE config C3 at full size: the two-class launch equals the
    one-kernel launch, and both equal the BVH-only kernel; most pixels are
    lean and really go to the lean kernel."""
    import torch
    ds = DeviceScene(scenes.mesh_bunny())
    _assert_same(_frames(ds, lambda f: _opts(1920, 1080, 16, f)), "C3")
    fb = torch.zeros(1920 * 1080 * 3, dtype=torch.float32, device="cuda")
    ds.render_device(_opts(1920, 1080, 16), fb)
    lean, general = ds.last_split()
    assert lean + general == 1920 * 1080 and lean > 0.8 * 1920 * 1080, (lean, general)
    batched, fallback = ds.last_batch()
    assert batched == general and 0 <= fallback < 0.05 * general, (batched, fallback, general)
    assert ds.last_lean_kernel() == 3 | 3 << 2  # the merged one-plane kernel
    ds.render_device(_opts(1920, 1080, 16, RT_FLAG_NO_MIX), fb)
    assert ds.last_lean_kernel() == 2 | 2 << 2  # the one-plane lean and general kernels
    ds.render_device(_opts(1920, 1080, 16, RT_FLAG_NO_LEAN1), fb)
    assert ds.last_lean_kernel() == 1 | 2 << 2
    ds.render_device(_opts(1920, 1080, 16, RT_FLAG_NO_GEN1), fb)
    assert ds.last_lean_kernel() == 2 | 1 << 2
    ds.render_device(_opts(1920, 1080, 16, RT_FLAG_NO_SPLIT), fb)
    assert ds.last_split() == (0, 1920 * 1080) and ds.last_lean_kernel() == 0


@pytest.mark.parametrize("m", [16, 32])
def test_lean1_kernel_choice(gpu, m):
    """k_render_lean1 / k_render_gen1 take the lean / general pixels of
    one-plane scenes at spp a multiple of 256 (m = 16, 32) with one or two
    distant lights; the general kernels take the others — frames equal
    either way (here and in the FLAG_SETS comparisons above)."""
    import torch
    one = scenes.mesh_bunny()
    one.lights = one.lights[:1]
    for scene, want in ((scenes.mesh_bunny(), 2 | 2 << 2), (one, 2 | 2 << 2), (_reflective_ground(False), 0)):
        ds = DeviceScene(scene)
        fb = torch.zeros(256 * 144 * 3, dtype=torch.float32, device="cuda")
        st = ds.render_device(_opts(256, 144, m, RT_FLAG_NO_MIX), fb)
        assert ds.last_lean_kernel() == want, (want, ds.last_lean_kernel())
        fb2 = torch.zeros_like(fb)
        st2 = ds.render_device(_opts(256, 144, m, RT_FLAG_NO_LEAN1 | RT_FLAG_NO_GEN1), fb2)
        assert st == st2 and torch.equal(fb, fb2)
    ds = DeviceScene(scenes.mesh_bunny())
    fb = torch.zeros(256 * 144 * 3, dtype=torch.float32, device="cuda")
    ds.render_device(_opts(256, 144, 8), fb)  # 64 spp: one iteration, no whole batch of 4
    assert ds.last_lean_kernel() == 1 | 1 << 2
    ds.render_device(_opts(256, 144, 16), fb)  # the merged kernel by default
    assert ds.last_lean_kernel() == 3 | 3 << 2


@pytest.mark.parametrize("dirs", [
    ((-2.0, -0.8, -0.3), (2.0, 0.8, -1.3)),   # opposite sides of the plane: one test per light
    ((-2.0, -0.8, -0.3), (2.0, 0.0, -1.3)),   # one parallel to it (no plane hit): per light
    ((-2.0, 0.0, -0.3), (2.0, 0.0, -1.3)),    # both parallel: the shared test
    ((-2.0, 0.0, -0.3),),                     # one light, parallel
    ((2.0, 0.8, -1.3),),                      # one light from below
    ("raw", (-2.0, -1.5, -0.3)),              # not normalised, |dir.y| > 1: per light
])
def test_lean1_light_sides(gpu, dirs):
    """k_render_lean1q / _mix1 test a lit sample's shadow rays against the
    plane once when every light is on the same side of it (or none off it,
    rtmi.cpp lights_one_side), per light otherwise: both equal the general
    kernels, frames and Stats."""
    import torch
    from rtmi.glm import normalize, vec
    from rtmi.scene import DistantLight
    s = scenes.mesh_bunny()
    raw = dirs[0] == "raw"
    s.lights = [DistantLight(color=vec3(1.0, 0.9, 0.8), intensity=3.0 - k, dir=vec(*d) if raw else normalize(vec(*d)))
                for k, d in enumerate(dirs[1:] if raw else dirs)]
    ds = DeviceScene(s)
    ref = torch.zeros(256 * 144 * 3, dtype=torch.float32, device="cuda")
    st_ref = ds.render_device(_opts(256, 144, 16, RT_FLAG_NO_LEAN1 | RT_FLAG_NO_GEN1), ref)
    for flags, kind in ((0, 3 | 3 << 2), (RT_FLAG_NO_MIX, 2 | 2 << 2)):
        fb = torch.zeros_like(ref)
        st = ds.render_device(_opts(256, 144, 16, flags), fb)
        assert ds.last_lean_kernel() == kind, (flags, ds.last_lean_kernel())
        assert st == st_ref and torch.equal(fb, ref), (dirs, flags, float((fb - ref).abs().max()))


@pytest.mark.parametrize("cam_y,bias", [(5.5, 1e-4), (5.5, 1e-7), (5.5, 0.0), (-3.0, 1e-4), (0.5, 1e-4)])
def test_lean1_camera_side_and_bias(gpu, cam_y, bias):
    """Camera above or below the ground plane and biases down to 0: every
    lean sample tests each light's shadow ray against the plane (round 3
    removed the host-proved shortcuts of lean modes 1 / 2), and the merged
    one-plane kernel renders the general kernels' frame and Stats."""
    import torch
    s = scenes.mesh_bunny()
    s.cameraToWorld = scenes._std_camera(0.0, cam_y, 1.5)
    ds = DeviceScene(s)
    ref = torch.zeros(256 * 144 * 3, dtype=torch.float32, device="cuda")
    st_ref = ds.render_device(_opts(256, 144, 16, RT_FLAG_NO_LEAN1 | RT_FLAG_NO_GEN1, bias=bias), ref)
    for flags in (0, RT_FLAG_NO_MIX):
        fb = torch.zeros_like(ref)
        st = ds.render_device(_opts(256, 144, 16, flags, bias=bias), fb)
        if flags == 0 and ds.last_split()[0] > 0:
            assert ds.last_lean_kernel() == 15, (cam_y, bias, ds.last_lean_kernel())  # k_render_mix1
        assert st == st_ref and torch.equal(fb, ref), (cam_y, bias, flags, float((fb - ref).abs().max()))


def test_no_split_without_records(gpu):
    """No lean kernel where no pixel can be lean: a point light (no skip
    bit), two meshes (no pixel records), fewer than 64 samples per pixel."""
    import torch
    for name, m in (("mesh_mix", 16), ("two_meshes", 16), ("bunny", 4)):
        ds = DeviceScene(SCENES[name]())
        fb = torch.zeros(200 * 120 * 3, dtype=torch.float32, device="cuda")
        ds.render_device(_opts(200, 120, m), fb)
        assert ds.last_split()[0] == 0, name


def test_batched_general_pixels_and_fallback(gpu):
    """The batched general kernel takes the general pixels of a one-mesh,
    distant-light scene and (almost) never falls back on the bunny; the fallback
    (forced by the test hook after a pixel's batches already ran) discards
    their colour and Stats — the frames above compare it bit for bit."""
    import torch
    ds = DeviceScene(scenes.mesh_bunny())
    fb = torch.zeros(320 * 180 * 3, dtype=torch.float32, device="cuda")
    ds.render_device(_opts(320, 180, 16), fb)
    lean, general = ds.last_split()
    batched, fallback = ds.last_batch()
    assert general > 0 and batched == general and 0 <= fallback < 0.01 * general, (general, batched, fallback)
    ds.render_device(_opts(320, 180, 16, RT_FLAG_BATCH_FALLBACK), fb)
    assert ds.last_batch() == (general, general)
    ds.render_device(_opts(320, 180, 16, RT_FLAG_NO_BATCH), fb)
    assert ds.last_batch()[0] == 0
    for name in ("mesh_mix", "two_meshes"):  # point light / two meshes: not batched
        d2 = DeviceScene(SCENES[name]())
        d2.render_device(_opts(200, 120, 16), fb)
        assert d2.last_batch()[0] == 0, name


def test_split_in_band_launches(gpu):
    """A multi-GPU rank's band set is a short launch: every launch — the
    first included, nothing is measured on an earlier frame (launch orders
    from measured costs are off by default, rtmi.cpp order_policy) — builds
    its own lean and general lists on the device and renders them. Same
    frames and Stats as the one-kernel launch."""
    import torch
    ds = DeviceScene(scenes.mesh_bunny())
    w, h, world = 640, 360, 8
    rows = band_rows(h, 4, world)
    for r in (0, 5):
        ref = torch.full((rows * w * 3,), -7.0, dtype=torch.float32, device="cuda")
        o_ref = Options(width=w, height=h, antialias=Antialias(akGrid, 16), bias=1e-4, precision=Precision.fp32,
                        flags=RT_FLAG_NO_SPLIT | RT_FLAG_NO_REORDER)
        st_ref = ds.render_bands_device(o_ref, ref, 4, r, world)
        o = Options(width=w, height=h, antialias=Antialias(akGrid, 16), bias=1e-4, precision=Precision.fp32)
        splits = []
        for _ in range(3):
            b = torch.full((rows * w * 3,), -7.0, dtype=torch.float32, device="cuda")
            st = ds.render_bands_device(o, b, 4, r, world)
            splits.append(ds.last_split())
            assert st == st_ref, (r, st, st_ref)
            assert torch.equal(b, ref), (r, float((b - ref).abs().max()))
        assert all(sp[0] > 0 and sp[1] > 0 for sp in splits) and len(set(splits)) == 1, splits
