"""The drop-in boundary exercised the way a maintainer would use it.

* tools/rv_render -- the C++ host driver over include/StateRender.hpp (the
  reference's class StateRender with drawCUDA's signature, ref_compat
  settings) -- runs on the GPU and its offscreen dump equals the oracle's
  frame (src/StateRender.cu:289-346, src/main.cpp:119-132);
* rv_bind_output: caller-owned pitched device images (pitch != W * bpp), as
  the reference renders into D3D12 placed footprints
  (src/CudaD3D12Texture.cu:215-306, src/StateRender.cu:247-252);
* rv_render_frames across a change of the caller stream's priority (the
  loop recreates only its streams; frames stay identical).
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import Hip

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def rv():
    import rvgrt_amd
    rvgrt_amd._lib.load()
    return rvgrt_amd


def _read_ppm(path):
    with open(path, "rb") as f:
        data = f.read()
    parts = data.split(b"\n", 3)
    assert parts[0] == b"P6"
    w, h = (int(v) for v in parts[1].split())
    return np.frombuffer(parts[3], np.uint8, w * h * 3).reshape(h, w, 3)


def test_cpp_facade_rv_render_matches_oracle(rv, oracle, atlas, tmp_path):
    """One reference frame (UpdateGIData + drawCUDA with ref_compat: time <-
    jitterY, jitter <- (0, 0), minDist's normalized-coordinate fetch) from the
    C++ tool, against the oracle."""
    exe = os.path.join(ROOT, "tools", "rv_render")
    assert os.path.exists(exe), "tools/rv_render not built (build())"
    out = tmp_path / "frame.ppm"
    pose = (110.0, 70.0, 120.0, 2.44, -3.4415927)
    W, H, lg = 256, 144, 7
    cmd = [exe, "--config", "c3", "--lg", str(lg), "--res", f"{W}x{H}", "--flags", "7", "--sweeps", "1",
           "--gi-per-frame", "1", "--warmup", "0", "--frames", "1", "--pose", ",".join(repr(v) for v in pose),
           "--atlas", os.path.join(ROOT, "rvgrt_amd", "assets", "texturepack.png"), "--out", str(out)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=180, cwd=ROOT)
    assert p.returncode == 0, p.stderr
    img = _read_ppm(out)
    # oracle: World build + 1 sweep (rv_gi_update 0), then UpdateGIData's first call = frame 0 over all
    # 32768 cells (RAYPS 262144 clipped), then drawCUDA
    ow = oracle.OracleWorld(lg, lg, lg, atlas=atlas).build(gi_sweeps=1)
    ow.gi_update(0, first=0, count=(1 << (lg - 2)) ** 3)
    cam = oracle.camera_from_pose(pose[:3], np.float32(pose[3]), np.float32(pose[4]), W, H)
    ref = oracle.render(ow, oracle.make_frame(W, H, 7 | oracle.F_REF_FETCH, cam))["rgba"][..., :3]
    assert np.array_equal(img, ref)


def test_bind_output_pitched_caller_buffers(rv, atlas):
    from rvgrt_amd.configs import TEST_POSES_128
    lg, W, H = 7, 200, 120
    hip = Hip()
    r = rv.StateRender((lg,) * 3, W, H, flags=rv.RV_FLAGS_REFERENCE, atlas=atlas)
    r.world_build()
    r.gi_update(0)
    cam, vp = rv.camera_from_pose(*TEST_POSES_128["P1"], W, H)
    r.frame(cam, vp)
    want = {k: r.readback(k).copy() for k in (rv.RV_IMAGE_COLOR, rv.RV_IMAGE_MOTION, rv.RV_IMAGE_DEPTH)}
    kinds = {rv.RV_IMAGE_COLOR: (4, 1024), rv.RV_IMAGE_MOTION: (4, 1088), rv.RV_IMAGE_DEPTH: (2, 576)}
    bufs = {}
    for k, (bpp, pitch) in kinds.items():
        assert pitch != W * bpp
        bufs[k] = hip.malloc(pitch * H)
        r.bind_output(k, bufs[k], pitch)
        p, pt = r.image_ptr(k)
        assert p == bufs[k] and pt == pitch
    with pytest.raises(rv.RvError):   # a pitch below the row size is refused
        r.bind_output(rv.RV_IMAGE_COLOR, bufs[rv.RV_IMAGE_COLOR], W * 4 - 4)
    r.frame(cam, vp)
    r.sync()
    for k, (bpp, pitch) in kinds.items():
        raw = hip.download2d(bufs[k], pitch, W * bpp, H)
        assert not raw[:, W * bpp:].any(), "bytes past the row were written"
        img = np.ascontiguousarray(raw[:, :W * bpp]).view(want[k].dtype).reshape(want[k].shape)
        assert np.array_equal(img, want[k]), k
        assert np.array_equal(r.readback(k), want[k]), k     # readback honours the bound pitch
    for k in kinds:                                          # NULL restores the library's own images
        r.bind_output(k, 0, 0)
    r.frame(cam, vp)
    assert np.array_equal(r.readback(rv.RV_IMAGE_COLOR), want[rv.RV_IMAGE_COLOR])
    r.close()
    hip.close()


def test_render_frames_across_stream_priority_change(rv, atlas):
    """rv_render_frames on a priority -1 stream, then a priority 0 stream, then
    -1 again: the loop's own streams are recreated, its batch buffers kept."""
    from rvgrt_amd.configs import TEST_POSES_128
    lg, W, H = 7, 320, 192
    hip = Hip()
    ref = rv.StateRender((lg,) * 3, W, H, flags=8, atlas=atlas)
    ref.world_build()
    cam, vp = rv.camera_from_pose(*TEST_POSES_128["P0"], W, H)
    ref.frame(cam, vp)
    want = ref.readback(rv.RV_IMAGE_COLOR).copy()
    r = rv.StateRender((lg,) * 3, W, H, flags=8, atlas=atlas)
    r.world_build()
    r.set_frames_in_flight(4)
    for prio in (-1, 0, -1):
        r.set_stream(hip.stream(prio))
        r.render_frames(9, cam, vp)
        assert np.array_equal(r.readback(rv.RV_IMAGE_COLOR), want), prio
    r.set_stream(0)
    r.close()
    ref.close()
    hip.close()
