#!/usr/bin/env python3
"""Speculative sphere steps, census first (CPU; the replay and rays of tools/sat_census.py).

approximateCSDF's step k+1 starts at p_{k+1} = p_k + dir * d(p_k) (src/raytracing_functions.cu:74-79),
so a chain of sphere steps is a chain of dependent gathers.  A lane that guesses d(p_k) = g before the
gather returns can gather d(p_k + dir * g) in the same round -- the candidate position is computed with
the same float operations as the real one, so where the guess is right the two-step advance is exact.
This census measures, on the longest lanes of the 64 longest pre-pass waves (the chains that end a
latency-bound launch) and on a random sample, how many gather rounds the chains would take with:
  * rep-m: guess "the last distance repeats", m steps deep (m extra gathers per round);
  * nbr-1: guess {g - 1, g, g + 1} one step deep (3 extra gathers per round); pair_up / pair_dn:
    {g, g + 1} / {g - 1, g}; *_afterT: no guesses before a march's step T (the long chains only).
DDA rounds (look-ahead groups, already one round per 8 steps) are counted unchanged.

usage: python tools/spec_census.py [config] [pose]      -> JSON on stdout
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sat_census import setup  # noqa: E402


def rounds_rep(seq, m):
    """Gather rounds of one sphere march under rep-m (the first step has no guess)."""
    n, j, r, g = len(seq), 0, 0, None
    while j < n:
        r += 1
        adv = 1
        if g is not None:
            while adv <= m and j + adv - 1 < n - 1 and seq[j + adv - 1] == g:
                adv += 1   # step j + adv - 1 read g: the gather at the next position was issued
        j += adv
        g = seq[j - 1]
    return r


def rounds_set(seq, cands, t0=0):
    """One step deep, guesses g + c for c in cands; no guessing before the march's step t0."""
    n, j, r, g = len(seq), 0, 0, None
    while j < n:
        r += 1
        adv = 2 if (g is not None and j >= t0 and j < n - 1 and (seq[j] - g) in cands) else 1
        j += adv
        g = seq[j - 1]
    return r


def rounds_nbr(seq):
    return rounds_set(seq, (-1, 0, 1))


def main():
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    pose = sys.argv[2] if len(sys.argv) > 2 else "P0"
    e = setup(cfg_name, pose)
    rp, solid, org, d, hit, o2, hit_index, sun = (e[k] for k in ("rp", "solid", "org", "d", "hit", "o2", "hit_index",
                                                                  "sun"))
    schemes = {"plain": lambda s: len(s), "rep1": lambda s: rounds_rep(s, 1), "rep2": lambda s: rounds_rep(s, 2),
               "rep4": lambda s: rounds_rep(s, 4), "nbr1": rounds_nbr,
               "pair_up": lambda s: rounds_set(s, (0, 1)), "pair_dn": lambda s: rounds_set(s, (-1, 0)),
               "rep1_after16": lambda s: rounds_set(s, (0,), 16), "nbr1_after16": lambda s: rounds_set(s, (-1, 0, 1), 16),
               "nbr1_after32": lambda s: rounds_set(s, (-1, 0, 1), 32)}

    def chain(i):
        recs = [rp.trace(solid, org[i], d[i])]
        if hit[i]:
            recs.append(rp.trace(solid, o2[hit_index[i]], sun, sun=True))
        out = {k: 0 for k in schemes}
        for a in recs:
            for k, f in schemes.items():
                out[k] += sum(f(s) for s in a["dseq"]) + a["dda_rounds"]
        out["dseq_head"] = [s[:40] for s in recs[0]["dseq"][:2]]
        return out

    res = {}
    for name, idx in (("top64_longest_lanes", e["lanes"]), ("random_3000", e["sample"][:1000])):
        ch = [chain(i) for i in idx]
        res[name] = {k: {"mean": float(np.mean([c[k] for c in ch])), "max": int(max(c[k] for c in ch))}
                     for k in schemes}
        if name.startswith("top"):
            res[name]["example_sequences"] = [c["dseq_head"] for c in ch[:3]]
    print(json.dumps({"config": cfg_name, "pose": pose, **res}, indent=1))


if __name__ == "__main__":
    main()
