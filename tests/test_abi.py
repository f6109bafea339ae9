"""The C-ABI library (librtmi.so) without a GPU: it loads, exports every
symbol include/rtmi.h declares with the struct layouts the header defines, and
its host-side entry points validate input and fail with codes, not aborts."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from rtmi import abi, glm, scenes
from rtmi._lib import LIB_PATH, lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "rtmi.h")


def header_functions():
    txt = open(HEADER).read()
    return set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(rt_\w+)\s*\(", txt, re.M))


def test_header_symbols_exported():
    names = header_functions()
    assert len(names) >= 15
    raw = C.CDLL(LIB_PATH)
    missing = [n for n in names if not hasattr(raw, n)]
    assert not missing, missing
    assert names == set(abi.SIGNATURES), names ^ set(abi.SIGNATURES)


def test_version_and_error_channel():
    L = lib()
    assert L.rt_version() == abi.RTMI_ABI_VERSION
    assert L.rt_scene_destroy(None) == abi.RT_E_INVALID
    assert b"null" in L.rt_last_error()


def test_library_built_from_these_sources():
    """Build provenance: librtmi.so carries the hash of the native sources it
    was compiled from (rt_build_source_hash, the Makefile computes it); a
    library left over from other sources fails here instead of being
    measured as if it were this tree's."""
    from rtmi._lib import kernel_source_hash, library_source_hash
    assert library_source_hash() == kernel_source_hash()


def test_no_gpu_is_an_error_not_a_crash():
    L = lib()
    if L.rt_device_count() > 0:
        pytest.skip("GPU present")
    assert L.rt_init(0) == abi.RT_E_DEVICE
    assert L.rt_last_error()


_LAYOUT_C = r"""
#include <stdio.h>
#include <stddef.h>
#include "rtmi.h"
#define S(t) printf(#t " %zu\n", sizeof(t));
#define O(t, f) printf(#t "." #f " %zu\n", offsetof(t, f));
int main(void) {
  S(rt_mesh_desc) S(rt_object_desc) S(rt_light_desc) S(rt_scene_desc) S(rt_options) S(rt_stats)
  S(rt_traversal_counters) S(rt_scene_info)
  O(rt_object_desc, world_to_object) O(rt_object_desc, radius) O(rt_object_desc, reflection)
  O(rt_light_desc, pos) O(rt_scene_desc, lights) O(rt_scene_desc, fov) O(rt_scene_desc, bg_color)
  O(rt_options, bias) O(rt_options, seed) O(rt_options, flags) O(rt_scene_info, build_ms)
  return 0;
}
"""


def test_struct_layouts_match_header(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(_LAYOUT_C)
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)],
                   check=True)
    out = dict(line.rsplit(" ", 1) for line in subprocess.check_output([str(exe)]).decode().split("\n")
               if line)
    for k, v in out.items():
        if "." in k:
            t, f = k.split(".")
            assert getattr(getattr(abi, t), f).offset == int(v), k
        else:
            assert C.sizeof(getattr(abi, k)) == int(v), k


def test_mat4_inverse_is_glm_inverse():
    L = lib()
    mats = [o.geometry.objectToWorld for o in scenes.boxes2().objects]
    mats.append(scenes.spheres_warm().cameraToWorld)
    for m in mats:
        a = (C.c_double * 16)(*glm.flat(m))
        out = (C.c_double * 16)()
        assert L.rt_mat4_inverse(a, out) == abi.RT_OK
        assert np.array_equal(np.array(out[:]), glm.flat(glm.inverse(m)))
    z = (C.c_double * 16)()
    assert L.rt_mat4_inverse(z, (C.c_double * 16)()) == abi.RT_E_INVALID


def test_load_geom_matches_reader(tmp_path):
    from rtmi.loaders import default_geom_path, readGeom
    L = lib()
    n = C.c_int64(0)
    p = default_geom_path().encode()
    assert L.rt_load_geom(p, C.byref(n), None) == abi.RT_OK
    assert n.value == 69451
    buf = np.zeros(n.value * 9, dtype=np.float64)
    assert L.rt_load_geom(p, C.byref(n), buf.ctypes.data_as(C.POINTER(C.c_double))) == abi.RT_OK
    assert np.array_equal(buf, readGeom(default_geom_path()).astype(np.float64).reshape(-1))
    # errors
    small = C.c_int64(10)
    assert L.rt_load_geom(p, C.byref(small), buf.ctypes.data_as(C.POINTER(C.c_double))) == abi.RT_E_INVALID
    assert L.rt_load_geom(str(tmp_path / "missing.geom").encode(), C.byref(n), None) == abi.RT_E_IO
    bad = tmp_path / "trunc.geom"
    bad.write_bytes(np.int32(5).tobytes() + b"\0" * 17)
    m = C.c_int64(5)
    assert L.rt_load_geom(str(bad).encode(), C.byref(m), buf.ctypes.data_as(C.POINTER(C.c_double))) == abi.RT_E_IO


def test_band_rows_matches_host_mapping():
    from rtmi.dist import band_rows
    L = lib()
    out = C.c_int32()
    for h, b, w in [(1080, 16, 1), (1080, 16, 8), (131, 7, 3), (1, 1, 8), (2160, 32, 4)]:
        assert L.rt_band_rows(h, b, w, C.byref(out)) == abi.RT_OK
        assert out.value == band_rows(h, b, w)
    assert L.rt_band_rows(0, 16, 1, C.byref(out)) == abi.RT_E_INVALID


def test_scene_create_validates_before_touching_a_device():
    from rtmi.scene import flatten
    L = lib()
    h = C.c_void_p()
    assert L.rt_scene_create(None, C.byref(h)) == abi.RT_E_INVALID
    s = scenes.spheres_warm(3)
    flat = flatten(s)
    flat._objs[0].type = 7
    assert L.rt_scene_create(C.byref(flat.desc), C.byref(h)) == abi.RT_E_INVALID
    flat = flatten(scenes.mesh_bunny())
    flat._objs[0].mesh = 3
    assert L.rt_scene_create(C.byref(flat.desc), C.byref(h)) == abi.RT_E_INVALID
    flat = flatten(scenes.spheres_warm(3))
    flat._objs[1].object_to_world[3] = 0.5  # projective row: unsupported
    assert L.rt_scene_create(C.byref(flat.desc), C.byref(h)) == abi.RT_E_UNSUPPORTED
    flat = flatten(scenes.mesh_bunny())
    flat.desc.bvh_builder = 9
    assert L.rt_scene_create(C.byref(flat.desc), C.byref(h)) == abi.RT_E_INVALID
    assert not h.value


def test_ppm_header_and_sizes():
    """rt_ppm_header / rt_ppm_payload_bytes (host-side, no GPU): writeHeader of
    framebuf.nim:60-61 and the payload size of the 8- / 16-bit formats."""
    import ctypes as C

    from rtmi._lib import lib
    L = lib()
    buf = C.create_string_buffer(64)
    n = L.rt_ppm_header(1920, 1080, 8, buf, 64)
    assert buf.raw[:n] == b"P6 1920 1080 255 "
    n = L.rt_ppm_header(4, 2, 16, buf, 64)
    assert buf.raw[:n] == b"P6 4 2 65535 "
    assert L.rt_ppm_header(4, 2, 8, buf, 5) < 0          # too small
    assert L.rt_ppm_payload_bytes(1920, 1080, 8) == 1920 * 1080 * 3
    assert L.rt_ppm_payload_bytes(3, 5, 16) == 3 * 5 * 6
    assert L.rt_ppm_payload_bytes(3, 5, 0) < 0 and L.rt_ppm_payload_bytes(3, 5, 17) < 0


def test_rgba_copy_matches_oracle(oracle_mod):
    """rtmi.framebuf.to_rgba (ImageRGBA.copyFrom, image.nim:45-54; the GPU
    pass's reference) equals the oracle's component on edge and random
    values, including the unclamped out-of-range cases."""
    from rtmi.framebuf import to_rgba
    rng = np.random.default_rng(11)
    v = np.concatenate([rng.random(20000).astype(np.float32) * 1.6 - 0.3,
                        np.array([0.0, -0.0, 0.5 / 255, 1.5 / 255, 254.5 / 255, 1.0, 1.002, 1.5, 2.0, -0.5 / 255,
                                  -0.3, 255.0, 1e7, -1e7, 1e30, -1e30, np.inf, -np.inf, np.nan], np.float32)])
    img = to_rgba(v.reshape(1, -1, 1).repeat(3, axis=2), alpha=0x7F)
    o = np.array([oracle_mod.rgba_component(float(x)) for x in v], np.uint8)
    assert np.array_equal(img[0, :, 0], o)
    assert np.array_equal(img[0, :, 2], o)
    assert (img[..., 3] == 0x7F).all()


def test_ppm_quantisation_matches_oracle(oracle_mod):
    """rtmi.framebuf.to_uint (the host writer and the GPU pass's reference)
    equals the oracle's outvalue on edge and random values."""
    import numpy as np

    from rtmi.framebuf import to_uint
    rng = np.random.default_rng(7)
    v = np.concatenate([rng.random(20000).astype(np.float32) * 1.4 - 0.2,
                        np.array([0.0031308, np.nextafter(np.float32(0.0031308), 1), 0.5 / 255, 1.5 / 255,
                                  254.5 / 255, 0.5, 1.0, -0.0, 2.0, -1.0, np.nan], np.float32)])
    for bits in (8, 16, 3):
        for srgb in (True, False):
            q = to_uint(v, bits, srgb).astype(np.int64)
            o = np.array([oracle_mod.ppm_outvalue(float(x), bits, srgb) for x in v])
            assert np.array_equal(q, o), (bits, srgb)
