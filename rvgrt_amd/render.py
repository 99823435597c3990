"""Host-side mirror of the reference's StateRender interface over the C ABI.

Reference: class StateRender (include/StateRender.cuh:11-47), its
drawCUDA (src/StateRender.cu:289-346), CoarseArray::InitializeGIData /
UpdateGIData (src/CoarseArray.cu:357-395) and the init sequence of
State::Create (src/State.cpp:24-56).  Every method forwards to
librvgrt_hip.so; errors raise RvError with rv_last_error().
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _lib
from ._lib import RvError, rv_camera, rv_config, rv_frame_desc, rv_hit, rv_stats


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def camera_from_pose(pos, yaw, pitch, width, height):
    """Character::Update basis + unjittered VP (src/Character.cpp:18-126)."""
    L = _lib.load()
    cam = rv_camera()
    vp = np.zeros(16, np.float32)
    st = L.rv_camera_from_pose(float(pos[0]), float(pos[1]), float(pos[2]), float(yaw),
                               float(pitch), int(width), int(height), C.byref(cam), _ptr(vp))
    if st != 0:
        raise RvError(f"rv_camera_from_pose: {_lib.STATUS_NAMES.get(st, st)}")
    return cam, vp


def frame_desc(cam: rv_camera, vp, prev_vp=None, time=0.0, jx=0.0, jy=0.0) -> rv_frame_desc:
    """One frame's inputs (rv_frame_desc): camera, unjittered VP and the
    previous frame's, effective time and jitter."""
    d = rv_frame_desc()
    d.cam = cam
    vp = np.ascontiguousarray(vp, np.float32)
    pvp = vp if prev_vp is None else np.ascontiguousarray(prev_vp, np.float32)
    for i in range(16):
        d.vp[i] = float(vp[i])
        d.prev_vp[i] = float(pvp[i])
    d.time, d.jitter_x, d.jitter_y = float(time), float(jx), float(jy)
    return d


def camera_dict(cam: rv_camera, vp):
    return {"pos": np.array(cam.pos[:], np.float32), "fo": np.array(cam.forward[:], np.float32),
            "ri": np.array(cam.right[:], np.float32), "up": np.array(cam.up[:], np.float32),
            "vp": np.asarray(vp, np.float32)}


def rccl_path():
    """The RCCL of the HIP runtime this process uses: torch's bundled librccl
    when torch is already imported (the library then shares torch's runtime),
    else None (the library loads the system librccl.so.1 next to the system
    HIP runtime it was linked with)."""
    import sys
    torch = sys.modules.get("torch")
    if torch is None:
        return None
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else None


class Comm:
    """RCCL communicator of one rank (rv_comm_*): rank 0 makes the unique id,
    the caller broadcasts its 128 bytes, every rank creates its side."""

    ID_BYTES = 128

    @staticmethod
    def unique_id(path=None) -> bytes:
        L = _lib.load()
        buf = (C.c_ubyte * Comm.ID_BYTES)()
        p = path if path is not None else rccl_path()
        st = L.rv_comm_unique_id(p.encode() if p else None, C.cast(buf, C.c_void_p), Comm.ID_BYTES)
        if st != 0:
            raise RvError(f"rv_comm_unique_id: {_lib.STATUS_NAMES.get(st, st)}")
        return bytes(buf)

    def __init__(self, render: "StateRender", uid: bytes, nranks: int, rank: int, path=None):
        self._L = _lib.load()
        buf = (C.c_ubyte * Comm.ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        p = path if path is not None else rccl_path()
        render._check(self._L.rv_comm_create(render._h, p.encode() if p else None, C.cast(buf, C.c_void_p),
                                             Comm.ID_BYTES, int(nranks), int(rank), C.byref(h)), "rv_comm_create")
        self._h = h
        self.rank, self.nranks = int(rank), int(nranks)

    @classmethod
    def loopback(cls, render: "StateRender", group: "LoopbackGroup", rank: int):
        """Rank `rank` of an in-process loopback group (rv_comm_create_loopback)."""
        self = cls.__new__(cls)
        self._L = _lib.load()
        h = C.c_void_p()
        render._check(self._L.rv_comm_create_loopback(render._h, group._h, group.nranks, int(rank), C.byref(h)),
                      "rv_comm_create_loopback")
        self._h = h
        self.rank, self.nranks = int(rank), group.nranks
        return self

    def wait(self, timeout_ms=0):
        """rv_comm_wait: bounded wait for this rank's loop; raises on a stalled peer."""
        st = self._L.rv_comm_wait(self._h, int(timeout_ms))
        if st != 0:
            raise RvError(f"rv_comm_wait: {_lib.STATUS_NAMES.get(st, st)}")

    def close(self):
        if getattr(self, "_h", None):
            self._L.rv_comm_destroy(self._h)
            self._h = None


class LoopbackGroup:
    """N in-process ranks on one GPU (rv_loopback_group_create)."""

    def __init__(self, nranks, timeout_ms=0):
        self._L = _lib.load()
        h = C.c_void_p()
        st = self._L.rv_loopback_group_create(int(nranks), int(timeout_ms), C.byref(h))
        if st != 0:
            raise RvError(f"rv_loopback_group_create: {_lib.STATUS_NAMES.get(st, st)}")
        self._h = h
        self.nranks = int(nranks)

    def close(self):
        if getattr(self, "_h", None):
            self._L.rv_loopback_group_destroy(self._h)
            self._h = None


class StateRender:
    """One render context on one GPU (reference: StateRender + its arrays)."""

    def __init__(self, log2_dims=(9, 9, 9), width=1920, height=1080, flags=_lib.RV_FLAGS_REFERENCE,
                 atlas=None, device=0, seed=(0, 0), ref_compat=True, ref_oob_jy=0.0,
                 gi_rays_per_frame=0, gi_init_saturate=False, tex_table=0, exits_off=0):
        self._L = _lib.load()
        self.width, self.height = int(width), int(height)
        self.log2_dims = tuple(int(v) for v in log2_dims)
        self.flags = int(flags)
        self._atlas = None if atlas is None else np.ascontiguousarray(atlas, np.uint8)
        cfg = rv_config()
        cfg.log2_x, cfg.log2_y, cfg.log2_z = self.log2_dims
        cfg.width, cfg.height, cfg.flags = self.width, self.height, self.flags
        cfg.seed_x, cfg.seed_z = int(seed[0]), int(seed[1])
        cfg.ref_compat, cfg.ref_oob_jy = int(bool(ref_compat)), float(ref_oob_jy)
        if self._atlas is not None:
            cfg.atlas_rgba8 = self._atlas.ctypes.data
            cfg.atlas_h, cfg.atlas_w = self._atlas.shape[0], self._atlas.shape[1]
        cfg.gi_rays_per_frame = int(gi_rays_per_frame)
        cfg.gi_init_saturate = int(bool(gi_init_saturate))
        cfg.tex_table, cfg.exits_off = int(tex_table), int(exits_off)
        h = C.c_void_p()
        st = self._L.rv_create(C.byref(cfg), int(device), C.byref(h))
        if st != 0:
            raise RvError(f"rv_create failed: {_lib.STATUS_NAMES.get(st, st)} "
                          "(needs a gfx950 GPU and a valid config)")
        self._h = h
        X, Y, Z = (1 << d for d in self.log2_dims)
        self.dims = (X, Y, Z)

    # ------------------------------------------------------------ plumbing
    def _check(self, st, what):
        if st != 0:
            msg = self._L.rv_last_error(self._h)
            raise RvError(f"{what}: {_lib.STATUS_NAMES.get(st, st)}: "
                          f"{msg.decode() if msg else ''}")

    def close(self):
        if getattr(self, "_h", None):
            self._L.rv_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, option, value):
        """rv_set_option (include/rvgrt.h): RV_OPT_* run-time options."""
        self._check(self._L.rv_set_option(self._h, int(option), int(value)), "rv_set_option")

    def get_option(self, option) -> int:
        v = C.c_int64()
        self._check(self._L.rv_get_option(self._h, int(option), C.byref(v)), "rv_get_option")
        return int(v.value)

    def set_stream(self, stream_handle: int):
        self._check(self._L.rv_set_stream(self._h, C.c_void_p(stream_handle)), "rv_set_stream")

    def set_frame_path(self, path):
        """RV_PATH_FUSED (per-pixel megakernels) or RV_PATH_WAVEFRONT (stage kernels)."""
        p = {"fused": _lib.RV_PATH_FUSED, "wavefront": _lib.RV_PATH_WAVEFRONT}.get(path, path)
        self._check(self._L.rv_set_frame_path(self._h, int(p)), "rv_set_frame_path")

    def set_frames_in_flight(self, n):
        """Frame slots for concurrent frames on alternating streams (fused path)."""
        self._check(self._L.rv_set_frames_in_flight(self._h, int(n)), "rv_set_frames_in_flight")

    def set_gi_async(self, on):
        self._check(self._L.rv_set_gi_async(self._h, int(bool(on))), "rv_set_gi_async")

    def set_pipeline(self, on):
        """rv_set_pipeline: pipelined reference frames in render_frames."""
        self._check(self._L.rv_set_pipeline(self._h, int(bool(on))), "rv_set_pipeline")

    def set_frame_group(self, n):
        """rv_set_frame_group: reference frames rendered n per launch (0 = off)."""
        self._check(self._L.rv_set_frame_group(self._h, int(n)), "rv_set_frame_group")

    def frame_group_effective(self):
        """The group size render_frames will use (0: per-frame pipeline)."""
        v = C.c_int32(0)
        self._check(self._L.rv_get_frame_group(self._h, C.byref(v)), "rv_get_frame_group")
        return int(v.value)

    def set_flow(self, on):
        """rv_set_flow: drop-in frames as one launch (pre-pass | next GI window | render)."""
        self._check(self._L.rv_set_flow(self._h, int(bool(on))), "rv_set_flow")

    def flow_info(self):
        """(active, launches, fallbacks) of the flow frames (rv_flow_info; synchronises)."""
        a, n, fb = C.c_int32(), C.c_uint64(), C.c_uint64()
        self._check(self._L.rv_flow_info(self._h, C.byref(a), C.byref(n), C.byref(fb)), "rv_flow_info")
        return bool(a.value), int(n.value), int(fb.value)

    def tex_table_info(self):
        """(active, bytes) of sampleTexture's tile table (rv_tex_table_info)."""
        a, n = C.c_int32(), C.c_uint64()
        self._check(self._L.rv_tex_table_info(self._h, C.byref(a), C.byref(n)), "rv_tex_table_info")
        return bool(a.value), int(n.value)

    def set_gi_stats(self, on):
        """rv_set_gi_stats: count the GI update's traversal steps (stage 'gi')."""
        self._check(self._L.rv_set_gi_stats(self._h, int(bool(on))), "rv_set_gi_stats")

    def sync(self):
        self._check(self._L.rv_sync(self._h), "rv_sync")

    # ------------------------------------------------------------ world
    def world_build(self):
        """State::Create: CArray::fill -> GenerateSDF -> InitializeGIData."""
        self._check(self._L.rv_world_build(self._h), "rv_world_build")

    def csdf_build(self):
        self._check(self._L.rv_csdf_build(self._h), "rv_csdf_build")

    def gi_init(self):
        self._check(self._L.rv_gi_init(self._h), "rv_gi_init")

    def gi_update(self, frame, first=0, count=None):
        if count is None:
            X, Y, Z = self.dims
            count = (X // 4) * (Y // 4) * (Z // 4)
        self._check(self._L.rv_gi_update(self._h, int(frame), int(first), int(count)), "rv_gi_update")

    def gi_sweeps(self, n):
        for s in range(n):
            self.gi_update(s)

    def update_gi_data(self):
        """CoarseArray::UpdateGIData: RAYPS cells, rolling offset."""
        self._check(self._L.rv_update_gi_data(self._h), "rv_update_gi_data")

    def world_import(self, kind, arr: np.ndarray):
        a = np.ascontiguousarray(arr)
        self._check(self._L.rv_world_import(self._h, kind, _ptr(a), a.nbytes), "rv_world_import")

    def world_export(self, kind) -> np.ndarray:
        X, Y, Z = self.dims
        if kind == _lib.RV_WORLD_BITS:
            a = np.zeros(X * Y * Z // 32, np.uint32)
        elif kind == _lib.RV_WORLD_CSDF:
            a = np.zeros(X * Y * Z // 8, np.uint8)
        else:
            a = np.zeros((X // 4) * (Y // 4) * (Z // 4) * 4, np.uint8)
        self._check(self._L.rv_world_export(self._h, kind, _ptr(a), a.nbytes), "rv_world_export")
        return a

    # ------------------------------------------------------------ frames
    def draw_cuda(self, pos, fo, up, ri, vp, prev_vp, jitter_x=0.0, jitter_y=0.0):
        """StateRender::drawCUDA, same argument order."""
        arrs = [np.ascontiguousarray(a, np.float32) for a in (pos, fo, up, ri, vp, prev_vp)]
        self._check(self._L.rv_draw_cuda(self._h, *[_ptr(a) for a in arrs],
                                         float(jitter_x), float(jitter_y)), "rv_draw_cuda")

    def frame(self, cam: rv_camera, vp, prev_vp=None, time=0.0, jx=0.0, jy=0.0, flags=None):
        vp = np.ascontiguousarray(vp, np.float32)
        pvp = vp if prev_vp is None else np.ascontiguousarray(prev_vp, np.float32)
        f = self.flags if flags is None else int(flags)
        self._check(self._L.rv_frame(self._h, C.byref(cam), _ptr(vp), _ptr(pvp), float(time),
                                     float(jx), float(jy), f), "rv_frame")

    def frame_tiles(self, cam, vp, tile_ids, tile_px=64, prev_vp=None, time=0.0, jx=0.0, jy=0.0,
                    flags=None):
        vp = np.ascontiguousarray(vp, np.float32)
        pvp = vp if prev_vp is None else np.ascontiguousarray(prev_vp, np.float32)
        ids = np.ascontiguousarray(tile_ids, np.int32)
        f = self.flags if flags is None else int(flags)
        self._check(self._L.rv_frame_tiles(self._h, C.byref(cam), _ptr(vp), _ptr(pvp), float(time),
                                           float(jx), float(jy), f, _ptr(ids), len(ids),
                                           int(tile_px)), "rv_frame_tiles")

    def set_tile_shard(self, tile_px, rank, nranks, root_weight=None):
        """This rank's interleaved share of T x T tiles for render_frames (0 ranks = full frames);
        root_weight = rank 0's share relative to the others (default 1)."""
        if root_weight is None:
            self._check(self._L.rv_set_tile_shard(self._h, int(tile_px), int(rank), int(nranks)), "rv_set_tile_shard")
        else:
            self._check(self._L.rv_set_tile_shard_weighted(self._h, int(tile_px), int(rank), int(nranks),
                                                           float(root_weight)), "rv_set_tile_shard_weighted")

    def set_gather_bpp(self, bpp):
        """Packed pixel bytes of the loop's tile gather (3 RGB24, 4 RGBA8)."""
        self._check(self._L.rv_set_gather_bpp(self._h, int(bpp)), "rv_set_gather_bpp")

    def render_frames(self, n, cam, vp, prev_vp=None, time=0.0, jx=0.0, jy=0.0, flags=None,
                      gi_per_frame=False, comm=None):
        """Native frame loop (rv_render_frames): n frames over the frame slots'
        streams; with a tile shard, this rank's tiles, the RCCL gather to rank 0
        and rank 0's untile every frame."""
        vp = np.ascontiguousarray(vp, np.float32)
        pvp = vp if prev_vp is None else np.ascontiguousarray(prev_vp, np.float32)
        f = self.flags if flags is None else int(flags)
        self._check(self._L.rv_render_frames(self._h, int(n), C.byref(cam), _ptr(vp), _ptr(pvp), float(time),
                                             float(jx), float(jy), f, int(bool(gi_per_frame)),
                                             comm._h if comm is not None else None), "rv_render_frames")

    def render_frame_seq(self, descs, next_desc=None, flags=None, gi_per_frame=False, comm=None):
        """rv_render_frame_seq: one rv_frame_desc per frame (moving camera,
        jitter/time sequence); next_desc = the frame after the sequence."""
        n = len(descs)
        arr = (rv_frame_desc * max(n, 1))(*descs)
        f = self.flags if flags is None else int(flags)
        nxt = C.byref(next_desc) if next_desc is not None else None
        self._check(self._L.rv_render_frame_seq(self._h, n, arr, nxt, f, int(bool(gi_per_frame)),
                                                comm._h if comm is not None else None), "rv_render_frame_seq")

    def tile_buffer(self):
        p, n = C.c_void_p(), C.c_size_t()
        self._check(self._L.rv_tile_buffer(self._h, C.byref(p), C.byref(n)), "rv_tile_buffer")
        return p.value, n.value

    def bind_tile_buffer(self, dev_ptr, nbytes):
        self._check(self._L.rv_bind_tile_buffer(self._h, C.c_void_p(dev_ptr), int(nbytes)),
                    "rv_bind_tile_buffer")

    def untile(self, dev_ptr: int, tile_ids, tile_px=64):
        ids = np.ascontiguousarray(tile_ids, np.int32)
        self._check(self._L.rv_untile(self._h, C.c_void_p(dev_ptr), _ptr(ids), len(ids), int(tile_px)),
                    "rv_untile")

    def bind_output(self, kind, dev_ptr, pitch):
        self._check(self._L.rv_bind_output(self._h, kind, C.c_void_p(dev_ptr), pitch), "rv_bind_output")

    def image_ptr(self, kind):
        p, pitch = C.c_void_p(), C.c_size_t()
        self._check(self._L.rv_image_ptr(self._h, kind, C.byref(p), C.byref(pitch)), "rv_image_ptr")
        return p.value, pitch.value

    def readback(self, kind=_lib.RV_IMAGE_COLOR) -> np.ndarray:
        W, H = self.width, self.height
        if kind == _lib.RV_IMAGE_COLOR:
            a = np.zeros((H, W, 4), np.uint8)
        elif kind == _lib.RV_IMAGE_MOTION:
            a = np.zeros((H, W, 2), np.uint16)
        elif kind == _lib.RV_IMAGE_DEPTH:
            a = np.zeros((H, W), np.uint16)
        else:
            a = np.zeros((H // 2, W // 2), np.float32)
        self._check(self._L.rv_readback(self._h, kind, _ptr(a), 0), "rv_readback")
        return a

    # ------------------------------------------------------------ test surface
    def trace_rays(self, org, dirs, dist) -> np.ndarray:
        org = np.ascontiguousarray(org, np.float32)
        dirs = np.ascontiguousarray(dirs, np.float32)
        dist = np.ascontiguousarray(dist, np.float32)
        n = len(dist)
        out = (rv_hit * max(n, 1))()
        self._check(self._L.rv_trace_rays(self._h, _ptr(org), _ptr(dirs), _ptr(dist), n,
                                          C.cast(out, C.c_void_p)), "rv_trace_rays")
        dt = np.dtype([("pos", "<f4", 3), ("normal", "<f4", 3), ("u", "<f4"), ("v", "<f4"),
                       ("hit", "<i4"), ("undef", "<i4"), ("sphere_steps", "<i4"),
                       ("dda_steps", "<i4"), ("csdf_checks", "<i4"), ("pad", "<i4")])
        return np.frombuffer(bytes(out), dt, count=n).copy()

    def stats(self, stage=-1) -> dict:
        """Counters (RV_F_STATS frames) of one RV_STAGE_* (-1 = all stages)."""
        s = rv_stats()
        self._check(self._L.rv_stats_stage(self._h, int(stage), C.byref(s)), "rv_stats_stage")
        return s.as_dict()

    def timing_enable(self, max_frames):
        self._check(self._L.rv_timing_enable(self._h, int(max_frames)), "rv_timing_enable")

    def timing_get(self):
        """(ms per stage [gi, prepass, render] summed over frames, frames)."""
        ms = (C.c_double * 3)()
        n = C.c_int32()
        self._check(self._L.rv_timing_get(self._h, ms, C.byref(n)), "rv_timing_get")
        return list(ms), n.value

    def timing_stages(self):
        """({stage name: summed ms}, frames) for the RV_STAGE_* slots."""
        n = len(_lib.STAGES)
        ms = (C.c_double * n)()
        k = C.c_int32()
        self._check(self._L.rv_timing_stages(self._h, ms, n, C.byref(k)), "rv_timing_stages")
        return dict(zip(_lib.STAGES, list(ms))), k.value

    def timing_launches(self):
        """{stage name: launches timed} (divide timing_stages' sums by these)."""
        n = len(_lib.STAGES)
        k = (C.c_int32 * n)()
        self._check(self._L.rv_timing_launches(self._h, k, n), "rv_timing_launches")
        return dict(zip(_lib.STAGES, list(k)))

    def stats_reset(self):
        self._check(self._L.rv_stats_reset(self._h), "rv_stats_reset")
