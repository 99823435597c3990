#!/usr/bin/env python3
"""Analyse an RV_WAVE_TRACE dump (variant build with -DRV_WAVE_TRACE): one
record of 8 dwords per k_render wave = t0 (2), t1 (2) in 100 MHz wall-clock
ticks, HW_ID, XCC_ID, tile bx, by.  Prints the kernel span, wave lifetime
distribution, per-XCD busy spans and the occupancy profile over time.

    python tools/wave_trace.py gpurun_out/wt_c2.bin
"""
import sys

import numpy as np


def main(path):
    a = np.fromfile(path, dtype=np.uint32).reshape(-1, 8)
    t0 = a[:, 0].astype(np.uint64) | (a[:, 1].astype(np.uint64) << 32)
    t1 = a[:, 2].astype(np.uint64) | (a[:, 3].astype(np.uint64) << 32)
    ok = t1 > 0
    a, t0, t1 = a[ok], t0[ok].astype(np.int64), t1[ok].astype(np.int64)
    base = t0.min()
    s, e = (t0 - base) * 10e-3, (t1 - base) * 10e-3          # microseconds
    life = e - s
    xcc = a[:, 5] & 0xF
    cu = (a[:, 4] >> 8) & 0xF
    sh = (a[:, 4] >> 12) & 1
    se = (a[:, 4] >> 13) & 0x7
    print(f"waves {len(a)}  span {e.max():.1f} us  (last start {s.max():.1f} us)")
    q = np.percentile(life, [0, 10, 50, 90, 99, 100])
    print("wave lifetime us  min/p10/p50/p90/p99/max:", " ".join(f"{v:.1f}" for v in q))
    print(f"sum of lifetimes {life.sum():.0f} wave-us;  mean {life.mean():.2f} us")
    for x in range(8):
        m = xcc == x
        if m.any():
            print(f"  XCD {x}: waves {m.sum():6d}  start {s[m].min():6.1f}  end {e[m].max():6.1f}  "
                  f"busy wave-us {life[m].sum():8.0f}")
    # resident waves over time (1 us bins)
    nb = int(np.ceil(e.max())) + 1
    occ = np.zeros(nb)
    for lo, hi in zip(s, e):
        occ[int(lo):int(hi) + 1] += 1
    print("resident waves per 10 us bin (chip):")
    for k in range(0, nb, 10):
        print(f"  {k:4d} us  {occ[k:k + 10].mean():8.0f}")
    # per-CU count of distinct slots as a sanity check
    slots = len(set(zip(xcc.tolist(), se.tolist(), sh.tolist(), cu.tolist())))
    print(f"distinct CUs seen: {slots}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/wt_c2.bin")
