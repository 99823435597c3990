#!/usr/bin/env python3
"""R9 sensitivity report (oracle/r9_study.py): every study variant against the
plain oracle on C1 whole, 128^3 and 256^3 reference frames (P0/P1).
Writes profiles/r03/r9_numerics.json and prints a table.

usage: python tools/r9_report.py [out.json]
       python tools/r9_report.py --long [out.json]   (the GI feedback loop over 64 UpdateGIData frames
                                                     -> profiles/r04/r9_long_gi.json)
       python tools/r9_report.py --drift [frames]    (128^3 P0 for 1024 frames, rendered every 64
                                                     -> profiles/r04/r9_long_gi_<frames>.json)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O                      # noqa: E402
from oracle import r9_study as S                    # noqa: E402
from rvgrt_amd.atlas import load_atlas              # noqa: E402
from rvgrt_amd.configs import CONFIGS, TEST_POSES_128, pose_f32   # noqa: E402

REF = O.F_PREPASS | O.F_WATER | O.F_GI


def cases():
    c1 = CONFIGS["c1"]
    yield "C1 256^3 640x360 primary P0", 8, 0, 640, 360, 0, pose_f32(c1, "P0")
    for p in ("P0", "P1"):
        yield f"128^3 320x180 reference {p}", 7, 1, 320, 180, REF, TEST_POSES_128[p]
    for p in ("P0", "P1"):
        pos, yaw, pitch = TEST_POSES_128[p]
        yield f"256^3 640x360 reference {p}", 8, 1, 640, 360, REF, (tuple(2 * v for v in pos), yaw, pitch)


def long_cases():
    for p in ("P0", "P1"):
        yield f"128^3 320x180 reference {p}", 7, 1, 320, 180, REF, TEST_POSES_128[p]
    pos, yaw, pitch = TEST_POSES_128["P1"]
    yield "256^3 640x360 reference P1", 8, 1, 640, 360, REF, (tuple(2 * v for v in pos), yaw, pitch)


def main_long(out_path):
    atlas = load_atlas()
    frames = 64
    report = {"generator": "tools/r9_report.py --long (oracle/r9_study.py long_gi_sequence)",
              "frames": frames, "rays_per_frame": 262144, "grazing_cos": S.GRAZING_COS, "cases": {}}
    for name, lg, sweeps, W, H, flags, pose in long_cases():
        t0 = time.time()
        curve = S.long_gi_sequence(lg, sweeps, frames, W, H, flags, pose, atlas,
                                   render_at=[1, 2, 4, 8, 16, 24, 32, 40, 48, 56, 64])
        report["cases"][name] = curve
        print(f"== {name}  ({time.time() - t0:.0f} s)", flush=True)
        for rec in curve:
            if "render" not in rec:
                continue
            line = f"  frame {rec['frame']:3d}  gi cells diff " + \
                   " ".join(f"{b} {v}" for b, v in rec["gi_cells_diff"].items())
            for b, m in rec["render"].items():
                line += (f" | {b}: exact {m['rgba_exact']:.5f} <=2LSB {m['rgba_le2']:.5f} hit {m['hit_agree']:.5f}"
                         f" tol {'ok' if S.tolerance_ok(m) else 'FAIL'}")
            print(line, flush=True)
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    with open(out_path, "w") as f:
        json.dump(report, f, indent=1)


def main_drift(frames):
    atlas = load_atlas()
    t0 = time.time()
    curve = S.long_gi_sequence(7, 1, frames, 320, 180, REF, TEST_POSES_128["P0"], atlas,
                               render_at=list(range(64, frames + 1, 64)))
    for rec in curve:
        if "render" in rec:
            print(rec["frame"], rec["gi_cells_diff"],
                  {b: (round(m["rgba_exact"], 5), round(m["rgba_le2"], 5), m["hit_agree"]) for b, m in rec["render"].items()},
                  flush=True)
    out = os.path.join(ROOT, "profiles", "r04", f"r9_long_gi_{frames}.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump({"generator": "tools/r9_report.py --drift", "case": "128^3 320x180 reference P0", "curve": curve}, f)
    print(f"done in {time.time() - t0:.0f} s")


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--drift":
        return main_drift(int(sys.argv[2]) if len(sys.argv) > 2 else 1024)
    if len(sys.argv) > 1 and sys.argv[1] == "--long":
        return main_long(sys.argv[2] if len(sys.argv) > 2 else
                         os.path.join(ROOT, "profiles", "r04", "r9_long_gi.json"))
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r03", "r9_numerics.json")
    atlas = load_atlas()
    report = {"generator": "tools/r9_report.py (oracle/r9_study.py)", "grazing_cos": S.GRAZING_COS,
              "cases": {}}
    for name, lg, sweeps, W, H, flags, pose in cases():
        t0 = time.time()
        wd, res = S.study(lg, sweeps, W, H, flags, pose, atlas)
        report["cases"][name] = {"world_diff": wd, "variants": res}
        print(f"== {name}  ({time.time() - t0:.0f} s)  world diffs: {wd}", flush=True)
        for v, m in res.items():
            print(f"  {v:22s} exact {m['rgba_exact']:.5f}  <=2LSB {m['rgba_le2']:.5f}  max {m['rgba_max']:3d}  "
                  f"hit {m['hit_agree']:.5f}  voxel {m['hit_voxel_agree']:.5f}  "
                  f"voxel(non-grazing) {m['hit_voxel_agree_nongrazing']:.5f}  "
                  f"tol {'ok' if S.tolerance_ok(m) else 'FAIL'}", flush=True)
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    with open(out_path, "w") as f:
        json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
