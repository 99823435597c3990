"""The C ABI library (librvgrt_hip.so) on a machine without a GPU: it loads,
exports every entry point include/rvgrt.h declares with the documented
status behaviour, and its host-only camera math matches the oracle."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    hdr = open(os.path.join(ROOT, "include", "rvgrt.h")).read()
    return re.findall(r"^\s*(?:rv_status|void|int32_t|const char\*)\s+(rv_\w+)\s*\(", hdr, re.M)


def test_library_exports_every_declared_symbol():
    from rvgrt_amd import _lib
    L = _lib.load()
    names = _declared()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # the Python binding covers every declared entry point too
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert set(names) <= bound, set(names) - bound


def test_abi_version_and_struct_sizes():
    from rvgrt_amd import _lib
    L = _lib.load()
    assert L.rv_abi_version() == 2   # 2: gi_init_saturate, tex_table, exits_off, rv_set_option
    assert C.sizeof(_lib.rv_config) == 72       # the C layout of include/rvgrt.h (pointer at offset 40)
    assert C.sizeof(_lib.rv_hit) == 56          # 8 floats + 6 int32
    assert C.sizeof(_lib.rv_stats) == 16 * 8
    assert C.sizeof(_lib.rv_camera) == 16 * 4


def test_invalid_config_rejected_without_touching_gpu():
    from rvgrt_amd import _lib
    L = _lib.load()
    cfg = _lib.rv_config()
    cfg.log2_x = cfg.log2_y = cfg.log2_z = 2      # too small
    cfg.width, cfg.height = 64, 64
    h = C.c_void_p()
    assert L.rv_create(C.byref(cfg), 0, C.byref(h)) == _lib.RV_ERR_INVALID
    cfg.log2_x = cfg.log2_y = cfg.log2_z = 6
    cfg.width = 1                                   # no half-res image (floor(W / 2) = 0)
    assert L.rv_create(C.byref(cfg), 0, C.byref(h)) == _lib.RV_ERR_INVALID
    cfg.width, cfg.height = 64, 32769               # images past 32-bit offsets
    assert L.rv_create(C.byref(cfg), 0, C.byref(h)) == _lib.RV_ERR_INVALID
    assert L.rv_frame(None, None, None, None, 0.0, 0.0, 0.0, 0) == _lib.RV_ERR_INVALID
    assert L.rv_destroy(None) is None


def test_create_fails_loudly_without_gfx950():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from rvgrt_amd import _lib
    L = _lib.load()
    cfg = _lib.rv_config()
    cfg.log2_x = cfg.log2_y = cfg.log2_z = 6
    cfg.width, cfg.height = 64, 64
    h = C.c_void_p()
    assert L.rv_create(C.byref(cfg), 0, C.byref(h)) == _lib.RV_ERR_NO_DEVICE
    import rvgrt_amd as rv
    with pytest.raises(rv.RvError):
        rv.StateRender((6, 6, 6), 64, 64)


@pytest.mark.parametrize("W,H", [(1920, 1080), (640, 360), (1280, 800)])
def test_camera_math_matches_oracle(oracle, W, H):
    """Character::Update basis + VP: host code in the library vs the oracle."""
    import rvgrt_amd as rv
    from rvgrt_amd.configs import CONFIGS, pose_f32
    for cfg in CONFIGS.values():
        pos, yaw, pitch = pose_f32(cfg)
        cam, vp = rv.camera_from_pose(pos, yaw, pitch, W, H)
        ref = oracle.camera_from_pose(pos, yaw, pitch, W, H)
        d = rv.camera_dict(cam, vp)
        for k in ("pos", "fo", "ri", "up", "vp"):
            assert np.array_equal(d[k].view(np.uint32), ref[k].view(np.uint32)), k
    # reference default pose (Character.cpp:30,45-46): forward points down ~17 deg
    cam, vp = rv.camera_from_pose((128, 350, 128), np.float32(-0.7), np.float32(-np.pi - 0.3), 1280, 800)
    fo = np.array(cam.forward[:])
    assert abs(fo[1] + np.sin(0.3)) < 1e-6 and abs(np.linalg.norm(fo) - 1) < 1e-6
    up = np.array(cam.up[:])
    assert up[1] < -0.9                               # "up" points to -Y (row 0 = top)
