"""Texture atlas decode (reference: src/Texturepack.cu:20-33 decodes
resources/texturepack.png with stb_image into 256x256 RGBA8, :63-120 uploads
it).  PNG is lossless, so an independent decoder (Pillow) must give the same
bytes as rvgrt_amd.atlas.decode_png; the asset must be the reference's file.
"""
import hashlib
import io

import numpy as np
import pytest

from rvgrt_amd import atlas as A

PIL = pytest.importorskip("PIL.Image")


def test_atlas_asset_is_reference_file():
    with open(A.ATLAS_PNG, "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == A.ATLAS_SHA256


def test_atlas_decode_matches_pillow():
    ours = A.load_atlas()
    theirs = np.asarray(PIL.open(A.ATLAS_PNG).convert("RGBA"))
    assert ours.shape == (256, 256, 4)
    assert np.array_equal(ours, theirs)


@pytest.mark.parametrize("mode", ["RGBA", "RGB"])
def test_decoder_all_filter_types(mode, tmp_path):
    """Pillow's optimising encoder picks filters 0-4 per row; our decoder
    must undo every one of them."""
    rng = np.random.default_rng(7)
    h, w = 37, 53
    img = rng.integers(0, 256, (h, w, 4 if mode == "RGBA" else 3), dtype=np.uint8)
    img[::3] = img[::3] // 7           # smooth rows favour sub/up/avg/paeth
    img[:, ::5] = 200
    buf = io.BytesIO()
    PIL.fromarray(img, mode).save(buf, format="PNG", optimize=True)
    dec = A.decode_png(buf.getvalue())
    want = np.asarray(PIL.open(io.BytesIO(buf.getvalue())).convert("RGBA"))
    assert np.array_equal(dec, want)


def test_write_png_roundtrip(tmp_path):
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (20, 31, 4), dtype=np.uint8)
    p = tmp_path / "x.png"
    A.write_png(str(p), img)
    assert np.array_equal(np.asarray(PIL.open(p).convert("RGBA")), img)
    assert np.array_equal(A.decode_png(p.read_bytes()), img)


def test_wrong_asset_rejected(monkeypatch, tmp_path):
    p = tmp_path / "other.png"
    A.write_png(str(p), np.zeros((4, 4, 4), np.uint8))
    monkeypatch.setattr(A, "ATLAS_PNG", str(p))
    monkeypatch.setattr(A, "_ATLAS_CACHE", None)
    with pytest.raises(ValueError):
        A.load_atlas()
