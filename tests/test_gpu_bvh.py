"""Device BVH builder (rt_scene_desc.bvh_builder = RT_BVH_PLOC,
csrc/rt_bvh_gpu.hip). Either tree must give the brute-force answer of
TriangleMesh.intersect (src/renderer/geom.nim:339-358: closest t, lowest face
on ties), so frames and Stats rendered through the PLOC tree must be
bit-identical to those through the host SAH tree, whose own parity with the
oracle test_gpu_parity.py pins — in both precisions, for meshes from 1 face to
the bunny, including degenerate ones (coincident faces, a flat grid)."""
import numpy as np
import pytest

from rtmi import Antialias, Options, Precision, akGrid, akNone, scenes
from rtmi.abi import RT_BVH_PLOC, RT_BVH_SAH
from rtmi.renderer import DeviceScene
from rtmi.scene import TriangleMesh

pytestmark = pytest.mark.gpu


def _soup(n, seed):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-2.0, 2.0, (n, 1, 3)) + np.array([0.0, 2.0, 0.0])
    v = (c + rng.normal(0.0, 0.6, (n, 3, 3))).reshape(-1, 3)
    return TriangleMesh(v, np.arange(3 * n, dtype=np.int32).reshape(-1, 3))


def _coincident():
    """64 copies of one face (equal Morton codes, exact t ties) plus 3 others."""
    base = np.array([[-1.0, 1.0, 0.0], [1.0, 1.0, 0.0], [0.0, 3.0, 0.0]])
    v = np.concatenate([np.tile(base, (64, 1)), base + [2.5, 0.0, 0.5], base + [-2.5, 0.0, -0.5],
                        base + [0.0, 0.5, 1.0]])
    return TriangleMesh(v, np.arange(len(v), dtype=np.int32).reshape(-1, 3))


def _flat_grid(k=32):
    """A k x k quad grid in the plane y = 1.5, facing the camera's side
    (zero-thickness boxes: zero half-areas in the SAH collapse)."""
    xs = np.linspace(-3.0, 3.0, k + 1)
    zs = np.linspace(-2.0, 2.0, k + 1)
    X, Z = np.meshgrid(xs, zs, indexing="ij")
    v = np.stack([X.ravel(), np.full(X.size, 1.5), Z.ravel()], 1)
    f = []
    for i in range(k):
        for j in range(k):
            a, b, c, d = i * (k + 1) + j, (i + 1) * (k + 1) + j, (i + 1) * (k + 1) + j + 1, i * (k + 1) + j + 1
            f += [[a, d, b], [b, d, c]]
    return TriangleMesh(v, np.array(f, np.int32))


def _scene(mesh):
    return scenes._mesh_scene(mesh, "m", (0.7, 0.6, 0.5))


CASES = {
    "one_face": lambda: _scene(_soup(1, 1)),
    "two_faces": lambda: _scene(_soup(2, 2)),
    "four_faces": lambda: _scene(_soup(4, 3)),
    "five_faces": lambda: _scene(_soup(5, 4)),
    "soup_300": lambda: _scene(_soup(300, 5)),
    "coincident": lambda: _scene(_coincident()),
    "flat_grid": lambda: _scene(_flat_grid()),
    "torus": lambda: _scene(scenes.torus_mesh(48, 24)),
    "mesh_mix": scenes.mesh_mix,
    "two_meshes": scenes.two_meshes,
}


def _render(ds, opts):
    import torch
    fb = torch.zeros(opts.height * opts.width * 3, dtype=torch.float32, device="cuda")
    st = ds.render_device(opts, fb)
    return fb, st


@pytest.mark.parametrize("name", list(CASES))
def test_ploc_tree_renders_identically(gpu, name):
    import torch
    scene = CASES[name]()
    a = DeviceScene(scene, bvh_builder=RT_BVH_SAH)
    b = DeviceScene(scene, bvh_builder=RT_BVH_PLOC)
    ia, ib = a.info(), b.info()
    assert ia["num_triangles"] == ib["num_triangles"]
    assert 1 <= ib["max_bvh_depth"] <= 60 and ib["num_bvh_nodes"] >= 1
    for opts in (Options(width=96, height=72, antialias=Antialias(akNone, 1), bias=1e-4, precision=Precision.fp64),
                 Options(width=160, height=120, antialias=Antialias(akGrid, 2), bias=1e-4,
                         precision=Precision.fp32)):
        fa, sa = _render(a, opts)
        fb, sb = _render(b, opts)
        assert sa == sb, (name, opts.precision)
        assert torch.equal(fa, fb), (name, opts.precision)


def test_ploc_bunny_identical_and_compact(gpu):
    import torch
    scene = scenes.mesh_bunny()
    a = DeviceScene(scene, bvh_builder=RT_BVH_SAH)
    b = DeviceScene(scene, bvh_builder=RT_BVH_PLOC)
    ia, ib = a.info(), b.info()
    # leaves of <= 4 faces: at least nf/4 leaves -> nf/4 - 1 inner nodes, and
    # a tree no more than 2x the SAH one
    assert ib["num_triangles"] // 4 - 1 <= ib["num_bvh_nodes"] <= 2 * ia["num_bvh_nodes"]
    opts = Options(width=320, height=180, antialias=Antialias(akGrid, 4), bias=1e-4, precision=Precision.fp32)
    fa, sa = _render(a, opts)
    fb, sb = _render(b, opts)
    assert sa == sb
    assert torch.equal(fa, fb)


def test_ploc_fp64_matches_oracle(gpu, oracle_mod):
    """Direct oracle check through the PLOC tree (float64: bit-exact)."""
    scene = scenes.mesh_mix()
    opts = Options(width=64, height=48, antialias=Antialias(akGrid, 2), bias=1e-4, precision=Precision.fp64)
    ds = DeviceScene(scene, bvh_builder=RT_BVH_PLOC)
    fb = np.zeros((48, 64, 3), np.float32)
    st = ds.render_lines(opts, fb, 0, 48)
    o = oracle_mod.OracleScene(scene)
    ref, rst, _ = o.render(opts)
    assert np.array_equal(fb, ref)
    assert st == rst


def test_bad_builder_rejected(gpu):
    from rtmi._lib import RtmiError
    with pytest.raises(RtmiError):
        DeviceScene(scenes.mesh_bunny(), bvh_builder=7)
