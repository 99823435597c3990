import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X)")


@pytest.fixture(scope="session")
def atlas():
    from rvgrt_amd.atlas import load_atlas
    return load_atlas()


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


_WORLD_CACHE = {}


@pytest.fixture(scope="session")
def oracle_world(oracle, atlas):
    """Factory: oracle world (lx, ly, lz, gi_sweeps, seed) built once per session."""
    def make(lx, ly, lz, gi_sweeps=1, seed=(0, 0)):
        key = (lx, ly, lz, gi_sweeps, seed)
        if key not in _WORLD_CACHE:
            w = oracle.OracleWorld(lx, ly, lz, atlas=atlas, ox=seed[0], oz=seed[1])
            _WORLD_CACHE[key] = w.build(gi_sweeps=gi_sweeps)
        return _WORLD_CACHE[key]
    return make


def random_rays(rng, n, dims, inside_frac=0.7):
    """Rays with origins inside / around the world, random directions incl.
    axis-aligned and zero components, start distances incl. negatives."""
    X, Y, Z = dims
    org = np.empty((n, 3), np.float32)
    k = int(n * inside_frac)
    org[:k] = rng.uniform(0, 1, (k, 3)) * np.array([X, Y, Z], np.float32)
    org[k:] = rng.uniform(-0.3, 1.3, (n - k, 3)) * np.array([X, Y, Z], np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    m = rng.uniform(size=n)
    d[m < 0.05, 0] = 0
    d[(m >= 0.05) & (m < 0.10), 1] = 0
    d[(m >= 0.10) & (m < 0.13)] *= np.array([0, 1, 0], np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True) + 1e-30
    d[np.linalg.norm(d, axis=1) == 0] = np.array([0, -1, 0], np.float32)
    dist = rng.uniform(-10, 40, n).astype(np.float32)
    dist[rng.uniform(size=n) < 0.3] = 0.0
    return org, d.astype(np.float32), dist


class Hip:
    """Streams and device buffers from the HIP runtime the library loaded
    (the test must not bring in a second runtime through torch)."""
    def __init__(self):
        import ctypes as C
        self.C = C
        self.L = C.CDLL("libamdhip64.so.7")
        self.owned = []

    def stream(self, priority=None):
        s = self.C.c_void_p()
        if priority is None:
            assert self.L.hipStreamCreate(self.C.byref(s)) == 0
        else:
            assert self.L.hipStreamCreateWithPriority(self.C.byref(s), 0, int(priority)) == 0
        self.owned.append(("s", s))
        return s.value

    def download2d(self, ptr, pitch, row_bytes, rows):
        """Copy a pitched device image to a host (rows, pitch) uint8 array."""
        import numpy as np
        out = np.zeros((rows, pitch), np.uint8)
        assert self.L.hipMemcpy(out.ctypes.data_as(self.C.c_void_p), self.C.c_void_p(ptr),
                                self.C.c_size_t(rows * pitch), 2) == 0   # hipMemcpyDeviceToHost
        return out

    def malloc(self, n):
        p = self.C.c_void_p()
        assert self.L.hipMalloc(self.C.byref(p), self.C.c_size_t(n)) == 0
        assert self.L.hipMemset(p, 0, self.C.c_size_t(n)) == 0
        self.owned.append(("m", p))
        return p.value

    def close(self):
        self.L.hipDeviceSynchronize()
        for kind, h in self.owned:
            (self.L.hipStreamDestroy if kind == "s" else self.L.hipFree)(h)
