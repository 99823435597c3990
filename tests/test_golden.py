"""The oracle against the committed golden fixtures (tests/golden/, made by
tests/golden/make_golden.py): world hashes, the six golden frames (RGBA8,
MV, depth hashes, PNGs and work counts) and the 256 golden rays.  Pins the
oracle itself against regressions; the GPU side of the same fixtures is in
tests/test_gpu_parity.py."""
import hashlib
import json
import os

import numpy as np

from rvgrt_amd.atlas import decode_png

GDIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_oracle_reproduces_golden_fixtures(oracle, oracle_world):
    g = json.load(open(os.path.join(GDIR, "golden.json")))
    for lg in (6, 7):
        w = oracle_world(lg, lg, lg, gi_sweeps=1)
        ref = g["worlds"][f"{1 << lg}^3"]
        assert sha(w.bits) == ref["bits"] and sha(w.csdf) == ref["csdf"]
        assert sha(w.gi) == ref["gi_after_1_sweep"]
    world = oracle_world(7, 7, 7, gi_sweeps=1)
    assert len(g["frames"]) == 6
    for key, fr in g["frames"].items():
        pos, yaw, pitch = fr["pose"]
        W, H = (int(v) for v in key.split("_")[1].split("x"))
        cam = oracle.camera_from_pose(pos, yaw, pitch, W, H)
        r = oracle.render(world, oracle.make_frame(W, H, fr["flags"], cam))
        assert sha(r["rgba"]) == fr["rgba"], key
        assert sha(r["mv"]) == fr["mv"] and sha(r["depth"]) == fr["depth"], key
        assert r["stats"] == fr["stats"], key
        with open(os.path.join(GDIR, f"{key}.png"), "rb") as f:
            assert np.array_equal(decode_png(f.read()), r["rgba"]), key
    t = np.load(os.path.join(GDIR, "traces_128.npz"))
    h = world.trace_batch(t["org"], t["dir"], t["dist"])
    for k in ("hit", "undef", "n_sphere", "n_dda", "n_check"):
        assert np.array_equal(h[k], t[k]), k
    assert np.array_equal(h["pos"].view(np.uint32), t["pos"].view(np.uint32))
    assert np.array_equal(h["normal"], t["normal"]) and np.array_equal(h["u"], t["u"])


def test_oracle_render_rows_equals_full_frame(oracle, oracle_world):
    """or_render_rows (the CPU baseline's stride-k row subsets) renders each
    listed row exactly as the whole-frame render does, with and without the
    pre-pass and the reference fetch."""
    from rvgrt_amd.configs import TEST_POSES_128
    world = oracle_world(7, 7, 7, gi_sweeps=1)
    W, H = 192, 108
    cam = oracle.camera_from_pose(*TEST_POSES_128["P0"], W, H)
    for flags in (0, oracle.F_SHADOW, 7, 7 | oracle.F_REF_FETCH):
        fr = oracle.make_frame(W, H, flags, cam)
        full = oracle.render(world, fr)
        rows = list(range(3, H, 16)) + [0, H - 1]
        sub = oracle.render_rows(world, fr, rows)
        for k in ("rgba", "mv", "depth"):
            assert np.array_equal(sub[k][rows], full[k][rows]), (flags, k)
        assert sub["stats"]["primary"] == W * len(rows)
