"""Whole-grid world fixtures at the full sizes (tests/golden/world_hashes.json,
made by tests/golden/make_world_hashes.py with the CPU oracle): helpers shared
by the GPU world tests and every full-size test that hands a GPU-built world
to the oracle."""
import hashlib
import json
import os

import numpy as np

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "world_hashes.json")
RAYPS = 262144

# benchmark config -> (world fixture, GI stage the config renders with)
CONFIG_WORLD = {"c2": ("c2", "gi_init"), "c3": ("c4", "gi_sweep1"), "c4": ("c4", "gi_sweep2"),
                "c5": ("c5", "gi_sweep2")}


def load():
    with open(PATH) as f:
        return json.load(f)["worlds"]


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def assert_grid(a: np.ndarray, rec: dict, what: str):
    """The array's sha256 equals the oracle's; on a mismatch, name the z-slabs
    (of rec['slabs']) that differ."""
    assert a.nbytes == rec["bytes"], (what, a.nbytes, rec["bytes"])
    if sha(a) == rec["sha256"]:
        return
    slabs = np.split(a.reshape(-1), len(rec["slabs"]))
    bad = [i for i, (s, h) in enumerate(zip(slabs, rec["slabs"])) if sha(s) != h]
    raise AssertionError(f"{what}: differs from the oracle's whole-grid build in z-slabs {bad} "
                         f"of {len(rec['slabs'])}")


def assert_world(r, rv, cfgname: str, gi=True, stage=None):
    """The GPU context's bits and CSDF (and, with gi, the GI grid of the
    config's sweeps, or of `stage`) equal the oracle's own whole-grid builds.
    cfgname: c2..c5, or a fixture name (c2, c4, c5, native) with `stage`."""
    name, cstage = CONFIG_WORLD.get(cfgname, (cfgname, None))
    stage = stage or cstage
    rec = load()[name]
    assert_grid(r.world_export(rv.RV_WORLD_BITS), rec["bits"], f"{name} bits")
    assert_grid(r.world_export(rv.RV_WORLD_CSDF), rec["csdf"], f"{name} csdf")
    if gi:
        assert_grid(r.world_export(rv.RV_WORLD_GI), rec[stage], f"{name} {stage}")
