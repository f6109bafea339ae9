"""Binned searches of the float32 kernel (csrc/rt_bins.h): camera rays test the
faces listed for their pixel, shadow rays to a distant light the faces listed
for their light-grid cell, instead of traversing the BVH. The lists are
conservative and the search keeps the BVH search's (t, face) key and shadow
early exit, so every frame and Stats count must be bit-identical to the
BVH-only kernel (RT_FLAG_NO_BINNING) — whose own parity with the oracle
test_gpu_parity.py pins."""
import numpy as np
import pytest

from rtmi import Antialias, Options, Precision, akGrid, akNone, scenes
from rtmi.abi import RT_FLAG_COUNT_TRAVERSAL, RT_FLAG_NO_BINNING
from rtmi.dist import band_rows
from rtmi.glm import Y_AXIS, X_AXIS, degToRad, inverse, mat4, rotate, scale, translate, vec3
from rtmi.renderer import DeviceScene
from rtmi.scene import TriangleMesh

pytestmark = pytest.mark.gpu


def _opts(w, h, m, flags=0, aa=akGrid):
    return Options(width=w, height=h, antialias=Antialias(aa, m), bias=1e-4, precision=Precision.fp32,
                   flags=flags)


def _render(ds, opts):
    import torch
    fb = torch.zeros(opts.height * opts.width * 3, dtype=torch.float32, device="cuda")
    st = ds.render_device(opts, fb)
    return fb, st


def _coincident():
    """64 copies of one face plus 3 others: exact (t, face) ties in every bin."""
    base = np.array([[-1.0, 1.0, 0.0], [1.0, 1.0, 0.0], [0.0, 3.0, 0.0]])
    v = np.concatenate([np.tile(base, (64, 1)), base + [2.5, 0.0, 0.5], base + [-2.5, 0.0, -0.5],
                        base + [0.0, 0.5, 1.0]])
    return TriangleMesh(v, np.arange(len(v), dtype=np.int32).reshape(-1, 3))


def _soup(n, seed):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-2.0, 2.0, (n, 1, 3)) + np.array([0.0, 2.0, 0.0])
    v = (c + rng.normal(0.0, 0.6, (n, 3, 3))).reshape(-1, 3)
    return TriangleMesh(v, np.arange(3 * n, dtype=np.int32).reshape(-1, 3))


def _rotated_torus():
    """A general object-to-world transform (rotation + non-uniform scale): the
    bins work in object space, the camera and light directions go through
    world_to_object."""
    mesh = scenes.torus_mesh(64, 32)
    m = translate(mat4(1.0), vec3(0.5, 1.2, -11.0))
    m = rotate(m, Y_AXIS, degToRad(35.0))
    m = rotate(m, X_AXIS, degToRad(-20.0))
    m = scale(m, vec3(1.3, 0.8, 1.1))
    mesh.objectToWorld = m
    mesh.worldToObject = inverse(m)
    return _placed_scene(mesh)


def _placed_scene(mesh):
    from rtmi.scene import Material, Object, Scene, initPlane
    objects = [Object("rot", mesh, Material(albedo=vec3(0.8, 0.7, 0.3))),
               Object("ground", initPlane(objectToWorld=mat4(1.0)), Material(albedo=vec3(0.4)))]
    return Scene(objects=objects, lights=scenes._warm_lights(), fov=50.0,
                 cameraToWorld=scenes._std_camera(0.0, 5.5, 1.5), bgColor=vec3(0.01, 0.03, 0.05))


CASES = {
    "bunny": scenes.mesh_bunny,
    "torus": lambda: scenes._mesh_scene(scenes.torus_mesh(96, 48), "t", (0.9, 0.5, 0.2)),
    "rotated_torus": _rotated_torus,
    "coincident": lambda: scenes._mesh_scene(_coincident(), "c", (0.7, 0.6, 0.5)),
    "soup_300": lambda: scenes._mesh_scene(_soup(300, 5), "s", (0.7, 0.6, 0.5)),
    # reflective mesh, point light (no grid: BVH), analytic objects after the
    # mesh (the shadow early exit's stop distance)
    "mesh_mix": scenes.mesh_mix,
    # two mesh objects: no face bins (BVH for every ray), object bins
    "two_meshes": scenes.two_meshes,
    # analytic scenes of 4..64 objects: object bins (per-pixel / per-cell
    # object masks), incl. rotated boxes (C2), reflections, a point light
    "boxes2": scenes.boxes2,
    "spheres_warm": scenes.spheres_warm,
    "spheres_reflection": scenes.spheres_reflection,
    "spheres_pointlight1": scenes.spheres_pointlight1,
}


@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("m", [4, 8, 16])
def test_bins_render_identically(gpu, name, m):
    import torch
    ds = DeviceScene(CASES[name]())
    fa, sa = _render(ds, _opts(200, 120, m))
    fb, sb = _render(ds, _opts(200, 120, m, RT_FLAG_NO_BINNING))
    assert sa == sb, (name, m)
    assert torch.equal(fa, fb), (name, m, float((fa - fb).abs().max()))


def test_bins_c3_full_frame_identical_and_used(gpu):
    """BASELINE config C3 at full size: bit-identical to the BVH-only frame,
    and the bins really replace most of the traversal (node fetches)."""
    import torch
    ds = DeviceScene(scenes.mesh_bunny())
    fa, sa = _render(ds, _opts(1920, 1080, 16))
    fb, sb = _render(ds, _opts(1920, 1080, 16, RT_FLAG_NO_BINNING))
    assert sa == sb
    assert torch.equal(fa, fb)
    _render(ds, _opts(1920, 1080, 16, RT_FLAG_COUNT_TRAVERSAL))
    binned = ds.last_counters()
    _render(ds, _opts(1920, 1080, 16, RT_FLAG_COUNT_TRAVERSAL | RT_FLAG_NO_BINNING))
    bvh = ds.last_counters()
    assert binned["wave_node_fetches"] < 0.2 * bvh["wave_node_fetches"], (binned, bvh)
    assert binned["wave_tri_fetches"] < bvh["wave_tri_fetches"], (binned, bvh)


def test_bins_bands_and_sizes(gpu):
    """Band launches (multi-GPU layout) and several image sizes (one pixel-list
    set per size, cached) match the BVH-only kernel."""
    import torch
    ds = DeviceScene(scenes.mesh_bunny())
    for w, h in ((320, 180), (257, 131), (320, 180)):
        for m in (4, 16):
            fa, sa = _render(ds, _opts(w, h, m))
            fb, sb = _render(ds, _opts(w, h, m, RT_FLAG_NO_BINNING))
            assert sa == sb and torch.equal(fa, fb), (w, h, m)
    rows = band_rows(180, 4, 3)
    for r in range(3):
        a = torch.zeros(rows * 320 * 3, dtype=torch.float32, device="cuda")
        b = torch.zeros_like(a)
        sa = ds.render_bands_device(_opts(320, 180, 8), a, 4, r, 3)
        sb = ds.render_bands_device(_opts(320, 180, 8, RT_FLAG_NO_BINNING), b, 4, r, 3)
        assert sa == sb and torch.equal(a, b), r


def test_bins_low_spp_falls_back(gpu):
    """Below 16 samples per pixel (a wave spans more than 4 pixels) camera
    rays keep the BVH; shadow rays still use the light grids."""
    import torch
    ds = DeviceScene(scenes.mesh_bunny())
    for aa, m in ((akNone, 1), (akGrid, 2)):
        fa, sa = _render(ds, _opts(240, 135, m, aa=aa))
        fb, sb = _render(ds, _opts(240, 135, m, RT_FLAG_NO_BINNING, aa=aa))
        assert sa == sb and torch.equal(fa, fb), m


def _planes_scene(wall):
    """The bunny over a tilted, rotated ground plane (general transform: the
    shadow skips' plane footprints go through it), optionally with a back
    wall (two planes: a pixel's rays may reach either)."""
    from rtmi.scene import Material, Object, Scene, initPlane
    mesh = scenes.baked_bunny()
    mesh.objectToWorld = translate(mat4(1.0), vec3(0.0, 0.0001, -12.0))
    mesh.worldToObject = inverse(mesh.objectToWorld)
    g = translate(mat4(1.0), vec3(0.0, -0.4, 0.0))
    g = rotate(g, X_AXIS, degToRad(4.0))
    g = rotate(g, Y_AXIS, degToRad(20.0))
    objects = [Object("bunny", mesh, Material(albedo=vec3(0.6, 0.9, 0.2))),
               Object("ground", initPlane(objectToWorld=g), Material(albedo=vec3(0.4)))]
    if wall:
        w = rotate(translate(mat4(1.0), vec3(0.0, 0.0, -24.0)), X_AXIS, degToRad(90.0))
        objects.append(Object("wall", initPlane(objectToWorld=w), Material(albedo=vec3(0.3, 0.3, 0.5))))
    return Scene(objects=objects, lights=scenes._warm_lights(), fov=50.0,
                 cameraToWorld=scenes._std_camera(0.0, 5.5, 1.5), bgColor=vec3(0.01, 0.03, 0.05))


@pytest.mark.parametrize("wall", [False, True])
def test_pixel_records_tilted_planes_and_bias(gpu, wall):
    """Pixel records (list length + shadow skips, rebuilt per bias) and the
    lean sample-loop instance over general-transform planes: bit-identical to
    the BVH-only kernel at two biases and two sample counts."""
    import torch
    ds = DeviceScene(_planes_scene(wall))
    for bias in (1e-4, 1e-2, 1e-4):
        for m in (8, 16):
            o = Options(width=320, height=180, antialias=Antialias(akGrid, m), bias=bias, precision=Precision.fp32)
            p = Options(width=320, height=180, antialias=Antialias(akGrid, m), bias=bias, precision=Precision.fp32,
                        flags=RT_FLAG_NO_BINNING)
            fa, sa = _render(ds, o)
            fb, sb = _render(ds, p)
            assert sa == sb, (wall, bias, m)
            assert torch.equal(fa, fb), (wall, bias, m, float((fa - fb).abs().max()))


@pytest.mark.parametrize("name", ["boxes2", "spheres_warm"])
@pytest.mark.parametrize("m", [8, 12, 16])
def test_object_batches_identical(gpu, name, m):
    """Analytic scenes with distant lights (C2): the object-binned batches (4
    samples per lane through the pixels' object masks and the shadow cells'
    masks) render the frame and Stats of the one-sample loop
    (RT_FLAG_NO_OBJ_BATCH) and of the unbinned kernel (RT_FLAG_NO_BINNING) —
    the same samples per lane in the same order (16 lanes per pixel at 64 spp,
    f32_lanes)."""
    import torch
    from rtmi.abi import RT_FLAG_NO_OBJ_BATCH
    ds = DeviceScene(CASES[name]())
    fa, sa = _render(ds, _opts(200, 120, m))
    for flags in (RT_FLAG_NO_OBJ_BATCH, RT_FLAG_NO_BINNING, RT_FLAG_NO_BINNING | RT_FLAG_NO_OBJ_BATCH):
        fb, sb = _render(ds, _opts(200, 120, m, flags))
        assert sa == sb, (name, m, flags)
        assert torch.equal(fa, fb), (name, m, flags, float((fa - fb).abs().max()))


def _boxes2_variant(kind):
    """boxes2 variants: scaled boxes and a non-uniformly scaled ball (the
    sphere test's `/ 2*a` quirk then scales t, geom.nim:215-233), low suns
    from other azimuths, two suns, a non-unit light direction."""
    from rtmi.glm import normalize, vec
    s = scenes.boxes2()
    if kind == "scaled":
        for i, o in enumerate(s.objects[1:], start=1):
            g = o.geometry
            f = vec3(2.0, 0.5, 1.0) if i == 2 else vec3(1.0 + 0.1 * (i % 4), 0.7 + 0.2 * (i % 3), 1.3)
            g.objectToWorld = scale(g.objectToWorld, f)
            g.worldToObject = inverse(g.objectToWorld)
        s.lights[0].dir = normalize(vec(-2.0, -0.35, 3.0))
    elif kind == "two_suns":
        s.lights[0].dir = normalize(vec(-4.0, -0.6, -1.0))
        s.lights.append(type(s.lights[0])(color=vec3(0.9, 0.8, 0.6), intensity=0.4,
                                          dir=normalize(vec(1.0, -0.2, 5.0))))
    elif kind == "nonunit":
        s.lights[0].dir = vec(3.0, -0.5, -4.0)
    return s


@pytest.mark.parametrize("kind", ["plain", "scaled", "two_suns", "nonunit"])
def test_object_batches_full_frame_variants(gpu, kind):
    """C2's full 1080p / 64 spp frame and variants of it: the object-binned
    batches' frames and Stats equal the one-sample loop's
    (RT_FLAG_NO_OBJ_BATCH), which test_gpu_configs.py pins to the oracle."""
    import torch
    from rtmi.abi import RT_FLAG_NO_OBJ_BATCH
    ds = DeviceScene(_boxes2_variant(kind))
    fa, sa = _render(ds, _opts(1920, 1080, 8))
    fb, sb = _render(ds, _opts(1920, 1080, 8, RT_FLAG_NO_OBJ_BATCH))
    assert sa == sb, (kind, sa, sb)
    assert torch.equal(fa, fb), (kind, float((fa - fb).abs().max()))


def test_counters_not_stale_after_no_stats_call(gpu):
    """rt_scene_last_counters after a call that set RT_FLAG_NO_STATS fails
    (that call reduced nothing) instead of returning the previous
    RT_FLAG_COUNT_TRAVERSAL call's counters (include/rtmi.h); a new counting
    call makes them readable again."""
    from rtmi._lib import RtmiError
    from rtmi.abi import RT_FLAG_NO_STATS
    ds = DeviceScene(scenes.mesh_bunny())
    _render(ds, _opts(160, 90, 8, RT_FLAG_COUNT_TRAVERSAL))
    first = ds.last_counters()
    assert first["lane_node_visits"] + first["lane_tri_tests"] > 0
    import torch
    fb = torch.zeros(160 * 90 * 3, dtype=torch.float32, device="cuda")
    ds.render_device(_opts(160, 90, 8, RT_FLAG_NO_STATS), fb, stats=False)
    with pytest.raises(RtmiError):
        ds.last_counters()
    _render(ds, _opts(160, 90, 8, RT_FLAG_COUNT_TRAVERSAL))
    assert ds.last_counters() == first
