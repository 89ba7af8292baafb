"""Dataset front-end (depth_sensor DATASET mode, depth_sensor.cpp:11-46, 186-196)
through the C-ABI, on the host: the PNG decoder against independent encodings
(PIL, and tests/pngw.py for interlaced / 16-bit colour / sub-byte / every
filter / split IDAT), OpenCV's imread conversions, the intr.txt parse and the
directory walk.  The reference ships no dataset (dataset/README.txt only), so
the frames here are synthetic."""
import os

import numpy as np
import pytest
from PIL import Image

import kfx
from pngw import opencv_color, write_png

RNG = np.random.default_rng(5)


def _arr(h, w, spp, bit, ctype, palette_n=0):
    hi = palette_n if ctype == 3 else (1 << bit)
    shape = (h, w) if spp == 1 else (h, w, spp)
    return RNG.integers(0, hi, size=shape, dtype=np.int64)


CASES = [  # (bit, ctype)
    (8, 0), (16, 0), (1, 0), (2, 0), (4, 0), (8, 2), (16, 2), (8, 4), (16, 4), (8, 6), (16, 6),
    (8, 3), (4, 3), (2, 3), (1, 3),
]


@pytest.mark.parametrize("interlace", [False, True])
@pytest.mark.parametrize("bit,ctype", CASES)
def test_png_decoder_matches_opencv_semantics(kfx_lib, tmp_path, bit, ctype, interlace):
    h, w = 13, 21  # odd sizes: partial bytes, empty Adam7 passes
    spp = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    pal = RNG.integers(0, 256, size=(1 << bit, 3)) if ctype == 3 else None
    img = _arr(h, w, spp, bit, ctype, palette_n=(1 << bit) if ctype == 3 else 0)
    p = str(tmp_path / "x.png")
    write_png(p, img, bit, ctype, interlace=interlace, palette=pal)
    assert kfx.png_info(p) == (w, h, spp, bit)
    assert np.array_equal(kfx.png_read_bgr8(p), opencv_color(img, bit, ctype, pal))
    if spp == 1 and ctype == 0:  # depth maps: one channel, values unchanged
        d = kfx.png_read_depth(p)
        ref = img.astype(np.float32) if bit >= 8 else (img * 255 // ((1 << bit) - 1)).astype(np.float32)
        assert np.array_equal(d, ref)


@pytest.mark.parametrize("mode", ["I;16", "L", "RGB", "RGBA", "P", "LA"])
def test_png_decoder_reads_pil_files(kfx_lib, tmp_path, mode):
    h, w = 48, 64
    p = str(tmp_path / "p.png")
    if mode == "I;16":
        a = RNG.integers(0, 65536, size=(h, w)).astype(np.uint16)
        Image.fromarray(a).save(p)  # uint16 -> mode I;16
        assert np.array_equal(kfx.png_read_depth(p), a.astype(np.float32))
        assert np.array_equal(kfx.png_read_bgr8(p)[:, :, 0], (a >> 8).astype(np.uint8))
        return
    if mode == "P":
        im = Image.fromarray(RNG.integers(0, 256, size=(h, w, 3)).astype(np.uint8)).convert("P")
        im.save(p)
        rgb = np.asarray(im.convert("RGB"))
    else:
        ch = {"L": 1, "RGB": 3, "RGBA": 4, "LA": 2}[mode]
        a = RNG.integers(0, 256, size=(h, w, ch)).astype(np.uint8)
        im = Image.fromarray(a[:, :, 0] if ch == 1 else a, mode=mode)
        im.save(p)
        rgb = np.asarray(im.convert("RGB"))  # alpha dropped, grey replicated
    assert np.array_equal(kfx.png_read_bgr8(p), rgb[:, :, ::-1])


def test_png_errors(kfx_lib, tmp_path):
    p = str(tmp_path / "e.png")
    write_png(p, _arr(8, 8, 1, 16, 0), 16, 0)
    good = open(p, "rb").read()
    for bad in (good[:40], good[:-20], b"GIF89a" + good[6:],
                good[:30] + bytes([good[30] ^ 1]) + good[31:]):  # truncated, truncated, signature, CRC
        open(p, "wb").write(bad)
        with pytest.raises(kfx.KfxError):
            kfx.png_read_depth(p)
    write_png(p, _arr(8, 8, 3, 8, 2), 8, 2)
    with pytest.raises(kfx.KfxError, match="one channel"):
        kfx.png_read_depth(p)
    with pytest.raises(kfx.KfxError):
        kfx.png_read_bgr8(str(tmp_path / "missing.png"))


def test_parse_intr_like_depth_sensor(kfx_lib, tmp_path):
    p = tmp_path / "intr.txt"
    p.write_text("525.0 0 319.5\n0 525.0 239.5\n0 0 1\n")
    assert kfx.parse_intr(str(p)) == pytest.approx((525.0, 319.5, 525.0, 239.5, 1.0))
    # values <= 0.1 are dropped wherever they are; a parse failure ends the reads
    p.write_text("600 0.05 320\n0.1 601 240\n0 0 1 7 8\n")
    assert kfx.parse_intr(str(p)) == pytest.approx((600, 320, 601, 240, 1))
    p.write_text("525 0 319.5\n0 525 x 239.5\n0 0 1\n")  # stops at 'x': 3 values only
    with pytest.raises(kfx.KfxError):
        kfx.parse_intr(str(p))
    with pytest.raises(kfx.KfxError):
        kfx.parse_intr(str(tmp_path / "none.txt"))


def _write_dataset(root, bgr, dep_u16, intr=True, names=None):
    os.makedirs(os.path.join(root, "color"))
    os.makedirs(os.path.join(root, "depth"))
    n = len(dep_u16)
    names = names or [f"{k:04d}.png" for k in range(n)]
    for k in range(n):
        Image.fromarray(np.ascontiguousarray(bgr[k][:, :, ::-1])).save(os.path.join(root, "color", names[k]))
        Image.fromarray(dep_u16[k]).save(os.path.join(root, "depth", names[k]))
    if intr:
        with open(os.path.join(root, "intr.txt"), "w") as f:
            f.write("525 0 159.5\n0 526 119.5\n0 0 1\n")


def test_dataset_directory(kfx_lib, tmp_path):
    n, h, w = 4, 24, 32
    bgr = RNG.integers(0, 256, size=(n, h, w, 3)).astype(np.uint8)
    dep = RNG.integers(0, 5000, size=(n, h, w)).astype(np.uint16)
    # names out of creation order: the reader sorts them (cv::glob)
    names = ["b.png", "a.png", "d.png", "c.png"]
    _write_dataset(str(tmp_path), bgr, dep, names=names)
    ds = kfx.Dataset(str(tmp_path))
    assert len(ds) == n and ds.has_intr
    it = ds.intrinsics
    assert (it.width, it.height) == (w, h)
    assert (it.fx, it.fy, it.cx, it.cy) == (525.0, 526.0, 159.5, 119.5)
    order = np.argsort(names)
    for k in range(n):
        c, d = ds.read(k)
        assert np.array_equal(c, bgr[order[k]]) and np.array_equal(d, dep[order[k]].astype(np.float32))
    with pytest.raises(kfx.KfxError):
        ds.read(n)
    ds.close()


def test_dataset_without_intr_or_frames(kfx_lib, tmp_path):
    bgr = RNG.integers(0, 256, size=(1, 8, 8, 3)).astype(np.uint8)
    dep = RNG.integers(0, 5000, size=(1, 8, 8)).astype(np.uint16)
    _write_dataset(str(tmp_path / "a"), bgr, dep, intr=False)
    ds = kfx.Dataset(str(tmp_path / "a"))
    assert not ds.has_intr and (ds.intrinsics.width, ds.intrinsics.height) == (640, 480)
    ds.close()
    os.makedirs(tmp_path / "empty" / "color")
    with pytest.raises(kfx.KfxError, match="no color"):
        kfx.Dataset(str(tmp_path / "empty"))
