"""ctypes mirror of include/rtmi.h (the C-ABI of librtmi.so).

The structs are shared by the product bindings (rtmi._lib) and by the test
oracle wrapper (oracle/oracle.py): one flattened scene description feeds both.
"""
import ctypes as C

RTMI_ABI_VERSION = 1

RT_OK = 0
RT_E_INVALID = -1
RT_E_UNSUPPORTED = -2
RT_E_DEVICE = -3
RT_E_NOMEM = -4
RT_E_IO = -5

RT_SPHERE, RT_PLANE, RT_BOX, RT_MESH = 0, 1, 2, 3
RT_DISTANT_LIGHT, RT_POINT_LIGHT = 0, 1
RT_AA_NONE, RT_AA_GRID, RT_AA_JITTERED, RT_AA_MULTI_JITTERED, RT_AA_CORRELATED_MULTI_JITTERED = range(5)
RT_FP32, RT_FP64 = 0, 1
RT_FLAG_ANYHIT_SHADOWS = 0x1
RT_FLAG_COUNT_TRAVERSAL = 0x2
RT_FLAG_NO_REORDER = 0x4
RT_FLAG_NO_BINNING = 0x8
RT_FLAG_NO_SPLIT = 0x10
RT_FLAG_NO_BATCH = 0x20
RT_FLAG_BATCH_FALLBACK = 0x40
RT_FLAG_NO_LEAN1 = 0x80
RT_FLAG_NO_GEN1 = 0x100
RT_FLAG_NO_STATS = 0x200
RT_FLAG_NO_MIX = 0x400
RT_FLAG_TIMING = 0x800
RT_FLAG_NO_OBJ_BATCH = 0x1000
RT_FLAG_COMPACT = 0x2000
RT_FLAG_F64_PER_LANE = 0x4000
RT_BVH_SAH = 0
RT_OBJ_SLASH_INDICES = 0x1
RT_BVH_PLOC = 1

_d16 = C.c_double * 16
_d3 = C.c_double * 3


class rt_mesh_desc(C.Structure):
    _fields_ = [
        ("vertices", C.POINTER(C.c_double)),
        ("num_vertices", C.c_int64),
        ("faces", C.POINTER(C.c_int32)),
        ("num_faces", C.c_int64),
        ("normals", C.POINTER(C.c_double)),
    ]


class rt_object_desc(C.Structure):
    _fields_ = [
        ("type", C.c_int32),
        ("mesh", C.c_int32),
        ("object_to_world", _d16),
        ("world_to_object", _d16),
        ("radius", C.c_double),
        ("box_min", _d3),
        ("box_max", _d3),
        ("albedo", _d3),
        ("reflection", C.c_double),
    ]


class rt_light_desc(C.Structure):
    _fields_ = [
        ("type", C.c_int32),
        ("reserved", C.c_int32),
        ("color", _d3),
        ("intensity", C.c_double),
        ("dir", _d3),
        ("pos", _d3),
    ]


class rt_scene_desc(C.Structure):
    _fields_ = [
        ("objects", C.POINTER(rt_object_desc)),
        ("num_objects", C.c_int32),
        ("num_lights", C.c_int32),
        ("lights", C.POINTER(rt_light_desc)),
        ("meshes", C.POINTER(rt_mesh_desc)),
        ("num_meshes", C.c_int32),
        ("bvh_builder", C.c_int32),
        ("fov", C.c_double),
        ("camera_to_world", _d16),
        ("bg_color", _d3),
    ]


class rt_options(C.Structure):
    _fields_ = [
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("aa_kind", C.c_int32),
        ("grid_size", C.c_int32),
        ("bias", C.c_double),
        ("max_ray_depth", C.c_int32),
        ("precision", C.c_int32),
        ("seed", C.c_uint64),
        ("flags", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


class rt_stats(C.Structure):
    _fields_ = [
        ("num_primary_rays", C.c_uint64),
        ("num_intersection_tests", C.c_uint64),
        ("num_intersection_hits", C.c_uint64),
        ("num_shadow_rays", C.c_uint64),
        ("num_reflection_rays", C.c_uint64),
    ]

    def as_dict(self):
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


class rt_response(C.Structure):
    _fields_ = [
        ("line", C.c_int32),
        ("status", C.c_int32),
        ("stats", rt_stats),
        ("error", C.c_char * 128),
    ]


RT_QUEUE_STOPPED, RT_QUEUE_RUNNING, RT_QUEUE_SHUTDOWN = 0, 1, 2


class rt_traversal_counters(C.Structure):
    _fields_ = [
        ("wave_node_fetches", C.c_uint64),
        ("wave_tri_fetches", C.c_uint64),
        ("lane_node_visits", C.c_uint64),
        ("lane_tri_tests", C.c_uint64),
    ]

    def as_dict(self):
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


class rt_scene_info(C.Structure):
    _fields_ = [
        ("num_objects", C.c_int64),
        ("num_lights", C.c_int64),
        ("num_meshes", C.c_int64),
        ("num_triangles", C.c_int64),
        ("num_bvh_nodes", C.c_int64),
        ("max_bvh_depth", C.c_int32),
        ("device", C.c_int32),
        ("device_bytes", C.c_int64),
        ("build_ms", C.c_double),
    ]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


# Every symbol include/rtmi.h declares, with its ctypes signature.
_P = C.c_void_p
SIGNATURES = {
    "rt_version": (C.c_int, []),
    "rt_build_source_hash": (C.c_char_p, []),
    "rt_last_error": (C.c_char_p, []),
    "rt_init": (C.c_int, [C.c_int]),
    "rt_device_count": (C.c_int, []),
    "rt_scene_create": (C.c_int, [C.POINTER(rt_scene_desc), C.POINTER(_P)]),
    "rt_scene_destroy": (C.c_int, [_P]),
    "rt_scene_get_info": (C.c_int, [_P, C.POINTER(rt_scene_info)]),
    "rt_scene_set_camera": (C.c_int, [_P, C.POINTER(C.c_double), C.c_double]),
    "rt_render_lines": (C.c_int, [_P, C.POINTER(rt_options), C.POINTER(C.c_float), C.c_int32,
                                  C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                  C.POINTER(rt_stats)]),
    "rt_render_lines_device": (C.c_int, [_P, C.POINTER(rt_options), _P, C.c_int32, C.c_int32,
                                         C.c_int32, C.c_int32, _P, C.POINTER(rt_stats)]),
    "rt_render_bands_device": (C.c_int, [_P, C.POINTER(rt_options), _P, C.c_int32, C.c_int32,
                                         C.c_int32, _P, C.POINTER(rt_stats)]),
    "rt_unshard_bands_device": (C.c_int, [_P, _P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P]),
    "rt_band_rows": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_int32)]),
    "rt_scene_last_counters": (C.c_int, [_P, C.POINTER(rt_traversal_counters)]),
    "rt_scene_last_split": (C.c_int, [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "rt_scene_last_lean_kernel": (C.c_int, [_P, C.POINTER(C.c_int32)]),
    "rt_scene_last_batch": (C.c_int, [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "rt_mat4_inverse": (C.c_int, [C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "rt_load_geom": (C.c_int, [C.c_char_p, C.POINTER(C.c_int64), C.POINTER(C.c_double)]),
    "rt_ppm_encode_device": (C.c_int, [_P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P, _P]),
    "rt_ppm_payload_bytes": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32]),
    "rt_rgba_encode_device": (C.c_int, [_P, C.c_int32, C.c_int32, C.c_uint8, _P, _P]),
    "rt_ppm_header": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_char_p, C.c_int32]),
    "rt_load_obj": (C.c_int, [C.c_char_p, C.c_uint32, C.POINTER(C.c_int64), C.POINTER(C.c_double),
                              C.POINTER(C.c_int64), C.POINTER(C.c_int32)]),
    "rt_write_geom": (C.c_int, [C.c_char_p, C.POINTER(C.c_double), C.c_int64, C.POINTER(C.c_int32), C.c_int64]),
    "rt_scene_last_stats": (C.c_int, [_P, C.POINTER(rt_stats)]),
    "rt_scene_last_timing": (C.c_int, [_P, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "rt_multi_create": (C.c_int, [C.POINTER(rt_scene_desc), C.POINTER(C.c_int32), C.c_int32, C.c_int32,
                                  C.POINTER(_P)]),
    "rt_render_frame_multi_device": (C.c_int, [_P, C.POINTER(rt_options), _P, C.POINTER(rt_stats)]),
    "rt_render_frame_multi": (C.c_int, [_P, C.POINTER(rt_options), C.POINTER(C.c_float), C.c_int32, C.c_int32,
                                        C.POINTER(rt_stats)]),
    "rt_multi_set_camera": (C.c_int, [_P, C.POINTER(C.c_double), C.c_double]),
    "rt_multi_destroy": (C.c_int, [_P]),
    "rt_queue_create": (C.c_int, [_P, C.POINTER(_P)]),
    "rt_queue_start": (C.c_int, [_P]),
    "rt_queue_stop": (C.c_int, [_P]),
    "rt_queue_state": (C.c_int, [_P]),
    "rt_queue_is_ready": (C.c_int, [_P]),
    "rt_queue_work": (C.c_int, [_P, C.POINTER(rt_options), C.POINTER(C.c_float), C.c_int32, C.c_int32,
                                C.c_int32, C.c_int32, C.c_int32]),
    "rt_queue_try_recv": (C.c_int, [_P, C.POINTER(rt_response)]),
    "rt_queue_pending": (C.c_int, [_P]),
    "rt_queue_reset": (C.c_int, [_P]),
    "rt_queue_shutdown": (C.c_int, [_P]),
    "rt_queue_destroy": (C.c_int, [_P]),
}


def bind(lib):
    """Attach argtypes/restype for every rtmi.h symbol; raise if one is missing."""
    missing = [n for n in SIGNATURES if not hasattr(lib, n)]
    if missing:
        raise ImportError(f"librtmi.so lacks exported symbols: {missing}")
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib
