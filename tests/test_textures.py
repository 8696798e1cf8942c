"""rt_image_load (Surface::LoadImage for PNG) against an independent encoder/decoder
(tests/pngref.py): every colour type, bit depth and row filter; the reference's earth.png."""
import os

import numpy as np
import pytest

import pngref

CASES = [  # (ctype, depth, channels)
    (0, 1, 1), (0, 2, 1), (0, 4, 1), (0, 8, 1), (0, 16, 1),
    (2, 8, 3), (2, 16, 3), (3, 1, 1), (3, 2, 1), (3, 4, 1), (3, 8, 1),
    (4, 8, 2), (4, 16, 2), (6, 8, 4), (6, 16, 4),
]


@pytest.mark.parametrize("ctype,depth,ch", CASES)
def test_png_decode_matches_independent_encoder(rt, tmp_path, ctype, depth, ch):
    rng = np.random.default_rng(ctype * 100 + depth)
    h, w = 11, 13
    hi = 1 << depth
    pal = None
    if ctype == 3:
        pal = rng.integers(0, 256, size=(hi, 3))
    samples = rng.integers(0, hi, size=(h, w, ch))
    f = tmp_path / "t.png"
    f.write_bytes(pngref.encode(samples, ctype, depth, palette=pal))
    got = rt.load_image(str(f))
    want = pngref.expected_pixels(samples, ctype, depth, palette=pal)
    assert got.shape == (h, w)
    assert np.array_equal(got, want)


def test_png_palette_with_transparency(rt, tmp_path):
    rng = np.random.default_rng(7)
    pal = rng.integers(0, 256, size=(16, 3))
    samples = rng.integers(0, 16, size=(5, 9, 1))
    f = tmp_path / "p.png"
    f.write_bytes(pngref.encode(samples, 3, 8, palette=pal, trns=[0] * 16))
    assert np.array_equal(rt.load_image(str(f)), pngref.expected_pixels(samples, 3, 8, palette=pal))


def test_png_errors(rt, tmp_path):
    with pytest.raises(rt.RTError) as e:
        rt.load_image(str(tmp_path / "missing.png"))
    assert e.value.code == rt.RT_ERR_IO
    bad = tmp_path / "bad.png"
    bad.write_bytes(b"not a png at all")
    with pytest.raises(rt.RTError):
        rt.load_image(str(bad))
    png = bytearray(pngref.encode(np.zeros((2, 2, 3), np.uint8), 2, 8))
    png[28] = 1   # IHDR interlace byte
    inter = tmp_path / "i.png"
    inter.write_bytes(bytes(png))
    with pytest.raises(rt.RTError) as e:
        rt.load_image(str(inter))
    assert e.value.code == rt.RT_ERR_UNSUPPORTED


def test_earth_png(rt, reference_assets):
    path = os.path.join(reference_assets, "earth.png")
    if not os.path.exists(path):
        pytest.skip("reference assets not present")
    img = rt.load_image(path)
    assert img.shape == (1024, 2048)    # power of two: TextureMaterial masks with w-1 / h-1
    assert np.array_equal(img[:24], pngref.decode_rgb8_rows(path, 24))
