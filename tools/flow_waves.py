#!/usr/bin/env python3
"""Per-wave timeline of one drop-in flow launch (k_ref_flow: pre-pass | next GI window | render, DESIGN.md
s5.1): where a renderLoop frame's time goes when it is latency-bound (C3 at 1080p: TD busy ~0.5).

Needs a library built with -DRV_PIPE_DIAG=1 (tools/build_variant.sh diag "-DRV_PIPE_DIAG=1", then
RVGRT_LIB=rvgrt_amd/variants/diag/librvgrt_hip.so); the context records its last flow launch's waves
(env RV_FLOW_WAVE_TRACE) and dumps them at rv_destroy.  Prints, per part, when its waves start and end
(us from the first wave's start), their lifetimes, the render waves' wait for their pre-pass tiles, and
the critical path: the last render waves to finish -- when they started, how long they waited, how long
they ran; and the pre-pass tiles of the longest waves, with the RV_FLOW_OPTS value that runs that tile's
wave alone (4: no GI or render part, 8: one pre-pass tile) -- its chain on an idle chip.  Not part of
the product.

usage: python tools/flow_waves.py [config] [pose] [frames] [--no-gi] [--static]
  --no-gi: renderLoop without its UpdateGIData calls, so the flow launches hold no GI window (an ablation:
           pre-pass + render).
  --static: every frame takes the first frame's camera (the same rays each launch: with one pre-pass tile
           alone, its chain runs on the caches the previous launch left, against a 1-frame run's cold one).  Every run also prints the mean k_ref_flow launch time over its frames (HIP
           events, after 8 warm-up frames) as MEAN_LAUNCH_US.
"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pct(v, qs=(50, 90, 99, 100)):
    return " ".join(f"p{q} {np.percentile(v, q):7.1f}" for q in qs)


def main():
    import torch
    import rvgrt_amd as rv
    from rvgrt_amd.atlas import load_atlas
    from rvgrt_amd.configs import CONFIGS, camera_path, pose_f32

    argv = [a for a in sys.argv[1:] if not a.startswith("--")]
    no_gi = "--no-gi" in sys.argv
    static = "--static" in sys.argv
    cfg = CONFIGS[argv[0] if len(argv) > 0 else "c3"]
    pose = argv[1] if len(argv) > 1 else "P0"
    nfr = int(argv[2]) if len(argv) > 2 else 40
    path = os.path.join(tempfile.gettempdir(), f"flow_waves_{os.getpid()}.bin")
    os.environ["RV_FLOW_WAVE_TRACE"] = path
    torch.cuda.set_device(0)
    W, H = cfg.width, cfg.height
    r = rv.StateRender((cfg.log2_n,) * 3, W, H, flags=cfg.flags, atlas=load_atlas())
    r.world_build()
    for s in range(max(cfg.gi_sweeps, 0)):
        r.gi_update(s)
    seq = camera_path(pose_f32(cfg, pose), W, H, nfr, pan=0.0005, ref_compat=True)
    for k in range(nfr):
        if k == 8:
            r.sync()
            r.timing_enable(2 * nfr + 2)
        d = seq[0] if static else seq[k]
        c = d.cam
        if not no_gi:
            r.update_gi_data()
        r.draw_cuda(c.pos[:], c.forward[:], c.up[:], c.right[:], np.ctypeslib.as_array(d.vp),
                    np.ctypeslib.as_array(d.vp if static else d.prev_vp), 0.0, d.time)
    r.sync()
    ms, _ = r.timing_stages()
    nl = r.timing_launches()
    mean_us = 1000.0 * ms["primary"] / nl["primary"] if nl["primary"] else 0.0
    r.close()
    raw = np.fromfile(path, np.uint32)
    os.unlink(path)
    lens, n = raw[:3].astype(int), int(raw[3])
    rec = raw[4:4 + 4 * n].reshape(n, 4).astype(np.int64)
    ok = rec[:, 0] != 0xFFFFFFFF            # padding workgroups leave their record unwritten? (they return early too)
    rec = rec[ok]
    t0 = rec[:, 1].min()
    start = (rec[:, 1] - t0) / 100.0        # 10-ns ticks -> us
    wait = (rec[:, 2] - t0) / 100.0
    end = (rec[:, 3] - t0) / 100.0
    part = rec[:, 0] & 0xFF
    tile = rec[:, 0] >> 8                   # pre-pass waves: bx | by << 12 (diagnostics builds)
    names = {1: "prepass", 0: "gi", 2: "render"}
    print(f"{cfg.name} {pose}: {W}x{H}, workgroups pre-pass {lens[0]}, GI {lens[1]}, render {lens[2]}; "
          f"launch span {end.max():.1f} us (last launch)")
    print(f"MEAN_LAUNCH_US {mean_us:.1f} over {nl['primary']} launches (RV_FLOW_OPTS={os.environ.get('RV_FLOW_OPTS', '0')}"
          f"{', no GI window' if no_gi else ''}{', static camera' if static else ''})")
    for q in (1, 0, 2):
        m = part == q
        if not m.any():
            continue
        life = end[m] - start[m]
        print(f"  {names[q]:8s} {m.sum():6d} waves  start {pct(start[m])}")
        print(f"  {'':8s} {'':12s}  end   {pct(end[m])}")
        print(f"  {'':8s} {'':12s}  life  {pct(life)}")
        if q == 2:
            print(f"  {'':8s} {'':12s}  wait  {pct(wait[m] - start[m])}")
            print(f"  {'':8s} {'':12s}  run   {pct(end[m] - wait[m])}")
    m = part == 2
    idx = np.flatnonzero(m)[np.argsort(-end[m])][:16]
    print("  last render waves to finish (start / tiles ready / end, us; run = end - ready):")
    for i in idx:
        print(f"    start {start[i]:7.1f}  ready {wait[i]:7.1f}  end {end[i]:7.1f}  run {end[i] - wait[i]:7.1f}")
    pp = part == 1
    top = np.flatnonzero(pp)[np.argsort(-(end[pp] - start[pp]))][:5]
    print("  longest pre-pass waves (tile bx, by: life us): " +
          ", ".join(f"{tile[i] & 0xFFF},{tile[i] >> 12}: {end[i] - start[i]:.1f}" for i in top))
    print(f"  LONGEST_TILE_OPTS {int((tile[top[0]] << 8) | 8 | 4)}")
    print(f"  pre-pass done at {end[pp].max():.1f} us; GI done at {end[part == 0].max() if (part == 0).any() else 0:.1f} us; "
          f"render waves dispatched from {start[m].min():.1f} us to {start[m].max():.1f} us")


if __name__ == "__main__":
    main()
