"""Texture loaders of the host mirror (host/fs_image.cpp) and their use by
the .scene material blocks (scene.cpp:276-306, material.cpp:63-95).

BMP follows bitmap.cpp:40-104, including its quirks: rows as stored
(bottom-up files are not flipped), BGR -> RGB / 255, the pixel data read
right after the 54 header bytes (off_bits ignored), 24-bit only, and a
truncated file leaving the map sized with zero texels.

EXR follows the LoadEXR() of the tinyexr header the reference vendors; the
files here come from tests/exrwrite.py, an independent encoder, so the
decoded values are known exactly. tinyexr's own test images are not part of
the reference, so parity with tinyexr itself is unpinned beyond the format.
"""
import struct

import numpy as np
import pytest

import exrwrite as X
import fsamd
import oracle_py
from descbuild import DescBuilder


def write_bmp(path, bgr_rows, bits=24, gap=0, truncate=0):
    h = len(bgr_rows)
    w = len(bgr_rows[0])
    stride = (w * 3 + 3) // 4 * 4
    data = b""
    for r in bgr_rows:
        line = bytes(np.asarray(r, np.uint8).ravel())
        data += line + b"\0" * (stride - w * 3)
    data = b"\xAB" * gap + data
    off = 54 + gap
    hdr = struct.pack("<2sIHHI", b"BM", off + len(data), 0, 0, off)
    hdr += struct.pack("<IiiHHIIiiII", 40, w, h, 1, bits, 0, len(data), 2835, 2835, 0, 0)
    blob = hdr + data
    if truncate:
        blob = blob[:-truncate]
    with open(path, "wb") as f:
        f.write(blob)


@pytest.mark.parametrize("w", [1, 2, 3, 4, 5])
def test_bmp_rows_padding_and_channel_order(tmp_path, w):
    rng = np.random.default_rng(w)
    rows = rng.integers(0, 256, (3, w, 3), dtype=np.uint8)
    p = tmp_path / "t.bmp"
    write_bmp(p, rows)
    ok, ww, hh, tex = fsamd.load_bitmap(p)
    assert ok and (ww, hh) == (w, 3)
    expect = (rows[:, :, ::-1].astype(np.float32) / np.float32(255.0)).ravel()  # BGR -> RGB, rows as stored
    np.testing.assert_array_equal(tex, expect)


def test_bmp_quirks(tmp_path):
    rows = np.arange(2 * 4 * 3, dtype=np.uint8).reshape(2, 4, 3)
    # off_bits is ignored: a gap between the headers and the pixels is read as pixels
    p = tmp_path / "gap.bmp"
    write_bmp(p, rows, gap=3)
    ok, w, h, tex = fsamd.load_bitmap(p)
    assert ok and tex[2] == np.float32(0xAB / 255.0)
    # only 24-bit files load
    p = tmp_path / "b32.bmp"
    write_bmp(p, rows, bits=32)
    ok, w, h, tex = fsamd.load_bitmap(p)
    assert not ok and tex.size == 0
    # a truncated file fails after sizing the map: texels of unread rows stay 0
    p = tmp_path / "trunc.bmp"
    write_bmp(p, rows, truncate=5)
    ok, w, h, tex = fsamd.load_bitmap(p)
    assert not ok and (w, h) == (4, 2) and tex.size == 24
    np.testing.assert_array_equal(tex[:12], (rows[0, :, ::-1].astype(np.float32) / np.float32(255.0)).ravel())
    assert not tex[12:].any()
    # a missing file loads nothing
    ok, w, h, tex = fsamd.load_bitmap(tmp_path / "missing.bmp")
    assert not ok and tex.size == 0


def _rgb(h, w, seed, kind):
    rng = np.random.default_rng(seed)
    a = rng.random((3, h, w), dtype=np.float32) * 8 - 2
    return a.astype(np.float16).astype(np.float32) if kind == X.HALF else a


@pytest.mark.parametrize("comp", [X.NONE, X.RLE, X.ZIPS, X.ZIP])
@pytest.mark.parametrize("kind", [X.HALF, X.FLOAT])
def test_exr_scanline(tmp_path, comp, kind):
    H, W = 37, 21
    r, g, b = _rgb(H, W, comp * 10 + kind, kind)
    p = tmp_path / "s.exr"
    X.write(p, [("B", kind, b), ("G", kind, g), ("R", kind, r)], compression=comp, origin=(5, -3))
    out = fsamd.load_exr(p)
    np.testing.assert_array_equal(out[..., 0], r)
    np.testing.assert_array_equal(out[..., 1], g)
    np.testing.assert_array_equal(out[..., 2], b)
    np.testing.assert_array_equal(out[..., 3], 1.0)  # no A channel


def test_exr_rle_runs_and_alpha(tmp_path):
    H, W = 9, 300  # long constant runs exercise the repeat branch
    r = np.zeros((H, W), np.float32)
    r[:, 100:] = 0.5
    g = np.full((H, W), 1.25, np.float32)
    b = np.linspace(0, 1, H * W, dtype=np.float32).reshape(H, W)
    a = np.full((H, W), 0.75, np.float32)
    p = tmp_path / "rle.exr"
    X.write(p, [("A", X.HALF, a), ("B", X.FLOAT, b), ("G", X.HALF, g), ("R", X.FLOAT, r)], compression=X.RLE)
    out = fsamd.load_exr(p)
    np.testing.assert_array_equal(out[..., 0], r)
    np.testing.assert_array_equal(out[..., 1], g)
    np.testing.assert_array_equal(out[..., 2], b)
    np.testing.assert_array_equal(out[..., 3], a)


def test_exr_decreasing_line_order_is_flipped(tmp_path):
    # tinyexr writes line y to row height-1-y when lineOrder is DECREASING_Y
    r, g, b = _rgb(6, 5, 3, X.FLOAT)
    p = tmp_path / "dec.exr"
    X.write(p, [("B", X.FLOAT, b), ("G", X.FLOAT, g), ("R", X.FLOAT, r)], line_order=1)
    out = fsamd.load_exr(p)
    np.testing.assert_array_equal(out[..., 0], r[::-1])


@pytest.mark.parametrize("comp", [X.NONE, X.ZIP])
def test_exr_tiled(tmp_path, comp):
    H, W = 19, 23
    r, g, b = _rgb(H, W, 11, X.HALF)
    p = tmp_path / "t.exr"
    X.write(p, [("B", X.HALF, b), ("G", X.HALF, g), ("R", X.HALF, r)], compression=comp, tiles=(8, 6))
    out = fsamd.load_exr(p)
    np.testing.assert_array_equal(out[..., :3], np.stack([r, g, b], -1))


def _piz_channels(H, W, seed, noisy):
    """A (UINT bits), B (smooth HALF), G (few HALF values), R (FLOAT; noisy:
    thousands of distinct 16-bit words, so the modulo 16-bit wavelet)."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W]
    b = (0.5 + 0.25 * np.sin(xx / 7.0) * np.cos(yy / 5.0)).astype(np.float32)
    g = (rng.integers(0, 40, (H, W)) / 8.0).astype(np.float32)
    if noisy:
        r = (rng.standard_normal((H, W)) * 3.0).astype(np.float32)
        a = rng.integers(0, 1 << 20, (H, W)).astype(np.uint32)
    else:
        r = (xx % 5 + yy // 3).astype(np.float32)  # small integers: the low 16-bit words are zero
        a = (xx // 3 + 100 * (yy // 4)).astype(np.uint32)
    return a, b, g, r


@pytest.mark.parametrize("tiles", [None, (16, 8), (32, 32)])
def test_exr_piz(tmp_path, tiles):
    """PIZ (tinyexr DecompressPiz, tiny_exr_loader.h:9303-9415): bitmap +
    reverse lookup table, Huffman with run lengths, 2D Haar wavelet on each
    16-bit layer (a FLOAT or UINT channel is two interleaved layers), 32-line
    scanline blocks (the last one ragged) or ragged tiles. The file comes
    from an independent encoder (tests/exrwrite.py), so the pixels are known."""
    H, W = 70, 45
    a, b, g, r = _piz_channels(H, W, 5, noisy=tiles is None)
    p = tmp_path / "piz.exr"
    X.write(p, [("A", X.UINT, a), ("B", X.HALF, b), ("G", X.HALF, g), ("R", X.FLOAT, r)], compression=X.PIZ,
            tiles=tiles)
    q = tmp_path / "none.exr"
    X.write(q, [("A", X.UINT, a), ("B", X.HALF, b), ("G", X.HALF, g), ("R", X.FLOAT, r)], tiles=tiles)
    if tiles != (16, 8):  # (16x8 tiles: the value bitmap outweighs 1.5 KB tiles, so they are stored raw)
        assert p.stat().st_size < q.stat().st_size  # compressed blocks, not stored ones
    out = fsamd.load_exr(p)
    np.testing.assert_array_equal(out[..., 0], r)
    np.testing.assert_array_equal(out[..., 1], g.astype(np.float16).astype(np.float32))
    np.testing.assert_array_equal(out[..., 2], b.astype(np.float16).astype(np.float32))
    np.testing.assert_array_equal(out[..., 3].view(np.uint32), a)  # UINT bits kept
    np.testing.assert_array_equal(out, fsamd.load_exr(q))


def test_exr_piz_small_and_stored_blocks(tmp_path):
    """Blocks whose PIZ form is not smaller are stored raw (tinyexr issue 40:
    equal sizes mean uncompressed); 1-pixel-wide and 1-line images take the
    wavelet's odd-column / odd-line paths only."""
    rng = np.random.default_rng(9)
    for H, W in ((1, 1), (1, 7), (9, 1), (3, 2)):
        r = rng.standard_normal((H, W)).astype(np.float32)
        p = tmp_path / f"s{H}x{W}.exr"
        X.write(p, [("B", X.FLOAT, r), ("G", X.FLOAT, r), ("R", X.FLOAT, r)], compression=X.PIZ)
        out = fsamd.load_exr(p)
        for c in range(3):
            np.testing.assert_array_equal(out[..., c], r)
    H, W = 32, 700  # > 16384 distinct 16-bit words in one block: the modulo (16-bit) wavelet
    yy, xx = np.mgrid[0:H, 0:W]
    r = (1.0 + 0.5 * np.cos(xx * 0.0091 - yy * 0.17)).astype(np.float32)  # smooth, full-precision mantissas
    g = (2.0 + np.sin(xx * 0.0137 + yy * 0.31)).astype(np.float32)
    words = np.concatenate([r.view(np.uint16).ravel(), g.view(np.uint16).ravel()])
    assert len(np.unique(words)) > 1 << 14
    p = tmp_path / "w16.exr"
    X.write(p, [("B", X.FLOAT, g), ("G", X.FLOAT, r), ("R", X.FLOAT, r)], compression=X.PIZ)
    assert p.stat().st_size < 0.9 * (H * W * 12)  # compressed, not stored
    out = fsamd.load_exr(p)
    np.testing.assert_array_equal(out[..., 0], r)
    np.testing.assert_array_equal(out[..., 2], g)
    H, W = 64, 33  # one constant channel next to noise: long zero runs after the first symbols
    r = np.full((H, W), 0.5, np.float32)
    g = rng.standard_normal((H, W)).astype(np.float32)
    p = tmp_path / "runs.exr"
    X.write(p, [("B", X.HALF, r), ("G", X.FLOAT, g), ("R", X.HALF, r)], compression=X.PIZ)
    out = fsamd.load_exr(p)
    np.testing.assert_array_equal(out[..., 0], r)
    np.testing.assert_array_equal(out[..., 1], g)


def test_exr_alpha_only_and_errors(tmp_path):
    a = np.arange(12, dtype=np.float32).reshape(3, 4)
    p = tmp_path / "a.exr"
    X.write(p, [("A", X.FLOAT, a)])
    out = fsamd.load_exr(p)
    for c in range(4):
        np.testing.assert_array_equal(out[..., c], a)
    p = tmp_path / "rg.exr"
    X.write(p, [("G", X.FLOAT, a), ("R", X.FLOAT, a)])
    with pytest.raises(fsamd.FsError, match="B channel not found"):
        fsamd.load_exr(p)
    with pytest.raises(fsamd.FsError):
        fsamd.load_exr(tmp_path / "missing.exr")


def test_scene_material_texture_blocks(tmp_path):
    """`texture` / `texture_scale` lines (scene.cpp:276-306) load the map into
    the material, and Scene::Describe hands it to the device description."""
    rows = np.random.default_rng(0).integers(0, 256, (4, 6, 3), dtype=np.uint8)
    write_bmp(tmp_path / "wood.bmp", rows)
    r, g, b = _rgb(3, 2, 1, X.FLOAT)
    X.write(tmp_path / "sky.exr", [("B", X.FLOAT, b), ("G", X.FLOAT, g), ("R", X.FLOAT, r)], compression=X.ZIP)
    scene = """material wood
{
  color 0.5 0.5 0.5
  texture_scale 0.25
  texture wood.bmp
}
material late_scale
{
  color 0.6 0.6 0.6
  texture wood.bmp
  texture_scale 2
}
material plain
{
  color 0.7 0.7 0.7
  texture None
}
material skymap
{
  emission 1 1 1
  texture sky.exr
}
sky
{
  material skymap
}
sphere
{
  material wood
  position 0 0 0
  radius 1
}
sphere
{
  material late_scale
  position 3 0 0
  radius 1
}
sphere
{
  material plain
  position 6 0 0
  radius 1
}
"""
    # ' texture %s' also matches the texture_scale line (scene.cpp:276): there
    # the name becomes "_scale" and late_scale ends up without a map.
    (tmp_path / "t.scene").write_text(scene)
    fsamd.reset_main_rng()
    s = fsamd.HostScene.load(str(tmp_path / "t.scene"))
    d = s.desc().contents
    assert d.num_textures == 2
    mats = [d.materials[i] for i in range(d.num_materials)]
    sky = d.materials[d.sky_material]
    assert sky.kind == fsamd.MAT_LIGHT and sky.texture >= 0
    objs = [d.objects[i] for i in range(d.num_objects)]
    wood, late, plain = (d.materials[o.material] for o in objs)
    assert wood.texture >= 0 and wood.texture != sky.texture
    assert wood.texture_scale == np.float32(0.25)
    assert late.texture < 0 and plain.texture < 0
    t = d.textures[wood.texture]
    assert (t.width, t.height) == (6, 4)
    got = np.ctypeslib.as_array(t.rgb, shape=(4 * 6 * 3,))
    np.testing.assert_array_equal(got, (rows[:, :, ::-1].astype(np.float32) / np.float32(255.0)).ravel())
    ts = d.textures[sky.texture]
    assert (ts.width, ts.height) == (2, 3)
    np.testing.assert_array_equal(np.ctypeslib.as_array(ts.rgb, shape=(18,)), np.stack([r, g, b], -1).ravel())


def test_oracle_samples_the_map():
    """The oracle's SampleDiffuse: a constant-colour map replaces diffuse_."""
    def render(with_map):
        b = DescBuilder()
        t = b.texture(np.full((4, 4, 3), 0.25, np.float32))
        light = b.material(fsamd.MAT_LIGHT, emissive=(2, 2, 2))
        b.sky = light
        m = b.material(fsamd.MAT_DIFFUSE, diffuse=(0.9, 0.9, 0.9), texture=t if with_map else -1)
        b.obj(fsamd.OBJ_PLANE, m, [0, 1, 0, 0])
        ptr = b.build()
        o = oracle_py.Scene(ptr)
        cam = fsamd.camera((0, 5, -10), (0, 0, 0), fov_y=40, aperture=0.0)
        f = o.render(cam, fsamd.render_params(8, 8, 2), threads=1)
        o.close()
        return f.color
    a, b = render(True), render(False)
    assert not np.array_equal(a, b)
    np.testing.assert_allclose(a, b * (0.25 / 0.9), rtol=1e-5)
