"""ctypes binding of the C ABI in include/rvgrt.h (librvgrt_hip.so).

The shared library is built in-tree by __graft_entry__.build() /
`make -C rvgrt_amd/csrc`.  There is no fallback: if the library (or a
gfx950 device) is missing, loading fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# RVGRT_LIB: an alternative build of the same library (A/B experiments)
LIB_PATH = os.environ.get("RVGRT_LIB") or os.path.join(_HERE, "librvgrt_hip.so")

RV_OK, RV_ERR_INVALID, RV_ERR_HIP, RV_ERR_OOM, RV_ERR_STATE, RV_ERR_NO_DEVICE = range(6)
RV_F_PREPASS, RV_F_WATER, RV_F_GI, RV_F_SHADOW, RV_F_STATS, RV_F_REF_FETCH = 1, 2, 4, 8, 16, 32
RV_FLAGS_REFERENCE = RV_F_PREPASS | RV_F_WATER | RV_F_GI
RV_IMAGE_COLOR, RV_IMAGE_MOTION, RV_IMAGE_DEPTH, RV_IMAGE_HALF_DIST, RV_IMAGE_HALF_SHADOW = range(5)
RV_WORLD_BITS, RV_WORLD_CSDF, RV_WORLD_GI = range(3)
RV_PATH_FUSED, RV_PATH_WAVEFRONT = 0, 1
# rv_set_option (include/rvgrt.h rv_option)
RV_OPT_PIPE_ORDER, RV_OPT_BATCH_STREAMS, RV_OPT_FLOW_SPIN, RV_OPT_FLOW_FORCE_FALLBACK, RV_OPT_GI_PAIRS, \
    RV_OPT_GI_SHARD_PROBE = range(1, 7)
# rv_config.exits_off bits
RV_EXIT_SKY, RV_EXIT_COLUMN, RV_EXIT_SUN = 1, 2, 4

STAGES = ["pp_primary", "pp_shadow", "primary", "shadow", "water", "cones", "shade", "gi"]
STATUS_NAMES = {0: "RV_OK", 1: "RV_ERR_INVALID", 2: "RV_ERR_HIP", 3: "RV_ERR_OOM",
                4: "RV_ERR_STATE", 5: "RV_ERR_NO_DEVICE"}


class rv_config(C.Structure):
    _fields_ = [("log2_x", C.c_int32), ("log2_y", C.c_int32), ("log2_z", C.c_int32),
                ("width", C.c_int32), ("height", C.c_int32), ("flags", C.c_int32),
                ("seed_x", C.c_int32), ("seed_z", C.c_int32),
                ("ref_compat", C.c_int32), ("ref_oob_jy", C.c_float),
                ("atlas_rgba8", C.c_void_p), ("atlas_w", C.c_int32), ("atlas_h", C.c_int32),
                ("gi_rays_per_frame", C.c_uint32), ("gi_init_saturate", C.c_int32),
                ("tex_table", C.c_int32), ("exits_off", C.c_int32)]


class rv_camera(C.Structure):
    _fields_ = [("pos", C.c_float * 3), ("forward", C.c_float * 3), ("right", C.c_float * 3),
                ("up", C.c_float * 3), ("mul", C.c_float * 2), ("add", C.c_float * 2)]


class rv_frame_desc(C.Structure):
    _fields_ = [("cam", rv_camera), ("vp", C.c_float * 16), ("prev_vp", C.c_float * 16),
                ("time", C.c_float), ("jitter_x", C.c_float), ("jitter_y", C.c_float)]


class rv_hit(C.Structure):
    _fields_ = [("pos", C.c_float * 3), ("normal", C.c_float * 3), ("u", C.c_float),
                ("v", C.c_float), ("hit", C.c_int32), ("undef", C.c_int32),
                ("sphere_steps", C.c_int32), ("dda_steps", C.c_int32),
                ("csdf_checks", C.c_int32), ("pad", C.c_int32)]


STAT_FIELDS = ["traces", "primary", "shadow", "refl", "refl_shadow", "prepass_primary",
               "prepass_shadow", "cones", "cone_steps", "sphere_steps", "dda_steps",
               "csdf_checks", "tex_samples", "undef_hits", "gi_traces", "frames"]


class rv_stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in STAT_FIELDS]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n in STAT_FIELDS}


# (name, restype, argtypes) for every entry point declared in include/rvgrt.h
P, I32, U32, U64, I64, F, SZ = (C.c_void_p, C.c_int32, C.c_uint32, C.c_uint64, C.c_int64,
                                C.c_float, C.c_size_t)
FP = C.POINTER(C.c_float)
SIGNATURES = [
    ("rv_abi_version", I32, []),
    ("rv_create", I32, [C.POINTER(rv_config), I32, C.POINTER(P)]),
    ("rv_destroy", None, [P]),
    ("rv_last_error", C.c_char_p, [P]),
    ("rv_set_stream", I32, [P, P]),
    ("rv_set_option", I32, [P, I32, C.c_int64]),
    ("rv_get_option", I32, [P, I32, C.POINTER(C.c_int64)]),
    ("rv_set_frame_path", I32, [P, I32]),
    ("rv_tile_shard_assign", I32, [I32, I32, I32, I32, C.c_float, P]),
    ("rv_set_gi_async", I32, [P, I32]),
    ("rv_set_pipeline", I32, [P, I32]),
    ("rv_set_frame_group", I32, [P, I32]),
    ("rv_get_frame_group", I32, [P, C.POINTER(C.c_int32)]),
    ("rv_set_flow", I32, [P, I32]),
    ("rv_tex_table_info", I32, [P, C.POINTER(C.c_int32), C.POINTER(C.c_uint64)]),
    ("rv_flow_info", I32, [P, C.POINTER(C.c_int32), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("rv_set_gi_stats", I32, [P, I32]),
    ("rv_set_frames_in_flight", I32, [P, I32]),
    ("rv_world_build", I32, [P]),
    ("rv_world_import", I32, [P, I32, P, SZ]),
    ("rv_world_export", I32, [P, I32, P, SZ]),
    ("rv_csdf_build", I32, [P]),
    ("rv_gi_init", I32, [P]),
    ("rv_gi_update", I32, [P, U32, U64, U64]),
    ("rv_update_gi_data", I32, [P]),
    ("rv_draw_cuda", I32, [P, P, P, P, P, P, P, F, F]),
    ("rv_frame", I32, [P, C.POINTER(rv_camera), P, P, F, F, F, I32]),
    ("rv_frame_tiles", I32, [P, C.POINTER(rv_camera), P, P, F, F, F, I32, P, I32, I32]),
    ("rv_tile_buffer", I32, [P, C.POINTER(P), C.POINTER(SZ)]),
    ("rv_bind_tile_buffer", I32, [P, P, SZ]),
    ("rv_untile", I32, [P, P, P, I32, I32]),
    ("rv_bind_output", I32, [P, I32, P, SZ]),
    ("rv_image_ptr", I32, [P, I32, C.POINTER(P), C.POINTER(SZ)]),
    ("rv_readback", I32, [P, I32, P, SZ]),
    ("rv_trace_rays", I32, [P, P, P, P, I64, P]),
    ("rv_camera_from_pose", I32, [F, F, F, F, F, I32, I32, C.POINTER(rv_camera), P]),
    ("rv_stats_get", I32, [P, C.POINTER(rv_stats)]),
    ("rv_stats_stage", I32, [P, I32, C.POINTER(rv_stats)]),
    ("rv_stats_reset", I32, [P]),
    ("rv_timing_enable", I32, [P, I32]),
    ("rv_timing_get", I32, [P, C.POINTER(C.c_double), C.POINTER(I32)]),
    ("rv_timing_stages", I32, [P, C.POINTER(C.c_double), I32, C.POINTER(I32)]),
    ("rv_timing_launches", I32, [P, C.POINTER(I32), I32]),
    ("rv_sync", I32, [P]),
    ("rv_comm_unique_id", I32, [C.c_char_p, P, SZ]),
    ("rv_comm_create", I32, [P, C.c_char_p, P, SZ, I32, I32, C.POINTER(P)]),
    ("rv_comm_destroy", None, [P]),
    ("rv_comm_wait", I32, [P, I32]),
    ("rv_loopback_group_create", I32, [I32, I32, C.POINTER(P)]),
    ("rv_loopback_group_destroy", None, [P]),
    ("rv_comm_create_loopback", I32, [P, P, I32, I32, C.POINTER(P)]),
    ("rv_set_tile_shard_weighted", I32, [P, I32, I32, I32, F]),
    ("rv_set_gather_bpp", I32, [P, I32]),
    ("rv_set_tile_shard", I32, [P, I32, I32, I32]),
    ("rv_render_frames", I32, [P, I32, C.POINTER(rv_camera), P, P, F, F, F, I32, I32, P]),
    ("rv_render_frame_seq", I32, [P, I32, C.POINTER(rv_frame_desc), C.POINTER(rv_frame_desc), I32, I32, P]),
]

_lib = None


def load() -> C.CDLL:
    """Load librvgrt_hip.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run __graft_entry__.build() "
                               "(make -C rvgrt_amd/csrc); there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            if os.environ.get("RVGRT_LIB") and not hasattr(L, name):
                continue   # an older experiment build: entry points it predates stay unbound
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


class RvError(RuntimeError):
    pass
