"""CPU checks of the file formats either side of the path:
the PNG / PGM / PFM readers behind EquirectangularMap::Load / PerspectiveMap::Load
(Depth.cpp:45-109, 277-355, 376-549; stb_image semantics: native channel count, 16-bit samples
/ 65535, 8-bit / 255), the Save16BitPNG writer (Depth.cpp:27-32), and the mode-0 LeReS layout
table of the C++ driver against pf_layouts (Main.cpp:788-843).  The PNGs are encoded here with
zlib + struct (all five filter types, palette, sub-byte gray) and decoded by the library; the
library's writer is decoded here.  No device calls."""
import ctypes as C
import os
import struct
import zlib

import numpy as np
import pytest

import panofuse
import pf_layouts as PL

LIB = os.path.join(os.path.dirname(panofuse.LIB_PATH), "libpanofuse_depth.so")
BIN = os.path.join(os.path.dirname(os.path.dirname(panofuse.LIB_PATH)), "bin", "panofuse_main")


@pytest.fixture(scope="module")
def lib():
    L = C.CDLL(LIB)
    fp = C.POINTER(C.c_float)
    ip = C.POINTER(C.c_int)
    L.pfd_load_map.argtypes = [C.c_char_p, C.c_int, fp, C.c_longlong, ip, ip, ip]
    L.pfd_save_png16.argtypes = [C.c_char_p, C.POINTER(C.c_uint16), C.c_int, C.c_int]
    L.pfd_leres_layout.argtypes = [fp, fp]
    L.pfd_save_jpeg.argtypes = [C.c_char_p, C.POINTER(C.c_uint8), C.c_int, C.c_int, C.c_int,
                                C.c_int, C.c_int]
    return L


def _load(lib, fn, is_emap=1):
    w, h, c = C.c_int(), C.c_int(), C.c_int()
    buf = np.zeros(1 << 22, np.float32)
    rc = lib.pfd_load_map(str(fn).encode(), is_emap, buf.ctypes.data_as(C.POINTER(C.c_float)),
                          buf.size, C.byref(w), C.byref(h), C.byref(c))
    if rc != 0:
        return None
    n = w.value * h.value * c.value
    return buf[:n].reshape(h.value, w.value, c.value)


def _chunk(t, d):
    return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return a if pa <= pb and pa <= pc else (b if pb <= pc else c)


def _filter_row(ft, row, prev, bpp):
    out = bytearray(len(row))
    for i in range(len(row)):
        a = row[i - bpp] if i >= bpp else 0
        b = prev[i] if prev is not None else 0
        c = prev[i - bpp] if (prev is not None and i >= bpp) else 0
        pred = [0, a, b, (a + b) >> 1, _paeth(a, b, c)][ft]
        out[i] = (row[i] - pred) & 0xFF
    return bytes(out)


def _png(path, rows, w, h, depth, ctype, plte=None, trns=None):
    """rows: list of raw (unfiltered) scanline bytes."""
    nc = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    bpp = max(1, nc * depth // 8)
    raw = b""
    prev = None
    for y, r in enumerate(rows):
        ft = y % 5
        raw += bytes([ft]) + _filter_row(ft, r, prev, bpp)
        prev = r
    data = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype,
                                                               0, 0, 0))
    if plte is not None:
        data += _chunk(b"PLTE", plte)
    if trns is not None:
        data += _chunk(b"tRNS", trns)
    data += _chunk(b"IDAT", zlib.compress(raw)) + _chunk(b"IEND", b"")
    open(path, "wb").write(data)


def test_png_gray16_and_rgb8_all_filters(lib, tmp_path):
    rng = np.random.default_rng(1)
    g16 = rng.integers(0, 65536, (13, 17), dtype=np.uint16)
    _png(tmp_path / "g16.png", [g16[y].astype(">u2").tobytes() for y in range(13)], 17, 13, 16, 0)
    got = _load(lib, tmp_path / "g16.png")
    assert got.shape == (13, 17, 1)
    np.testing.assert_array_equal(got[..., 0], g16.astype(np.float32) / np.float32(65535.0))
    rgb = rng.integers(0, 256, (9, 11, 3), dtype=np.uint8)
    _png(tmp_path / "rgb.png", [rgb[y].tobytes() for y in range(9)], 11, 9, 8, 2)
    got = _load(lib, tmp_path / "rgb.png", 0)
    assert got.shape == (9, 11, 3)
    np.testing.assert_array_equal(got, rgb.astype(np.float32) / np.float32(255.0))
    rgba16 = rng.integers(0, 65536, (5, 7, 4), dtype=np.uint16)
    _png(tmp_path / "rgba16.png", [rgba16[y].astype(">u2").tobytes() for y in range(5)], 7, 5,
         16, 6)
    got = _load(lib, tmp_path / "rgba16.png")
    np.testing.assert_array_equal(got, rgba16.astype(np.float32) / np.float32(65535.0))


def test_png_palette_and_subbyte_gray(lib, tmp_path):
    plte = bytes(range(30))  # 10 entries
    idx = np.arange(24).reshape(4, 6) % 10
    rows = []
    for y in range(4):  # 4-bit indices, two per byte
        r = idx[y]
        rows.append(bytes((int(r[i]) << 4) | int(r[i + 1]) for i in range(0, 6, 2)))
    _png(tmp_path / "pal.png", rows, 6, 4, 4, 3, plte=plte)
    got = _load(lib, tmp_path / "pal.png")
    assert got.shape == (4, 6, 3)
    pal = np.frombuffer(plte, np.uint8).reshape(10, 3)
    np.testing.assert_array_equal(got, pal[idx].astype(np.float32) / np.float32(255.0))
    bits = np.random.default_rng(2).integers(0, 2, (3, 10))
    rows = [np.packbits(bits[y]).tobytes() for y in range(3)]
    _png(tmp_path / "g1.png", rows, 10, 3, 1, 0)
    got = _load(lib, tmp_path / "g1.png")
    np.testing.assert_array_equal(got[..., 0], bits.astype(np.float32) * 255 / np.float32(255.0))


def _read_png16(path):
    d = open(path, "rb").read()
    assert d[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat = 8, b""
    while pos < len(d):
        n = struct.unpack(">I", d[pos:pos + 4])[0]
        t = d[pos + 4:pos + 8]
        body = d[pos + 8:pos + 8 + n]
        assert struct.unpack(">I", d[pos + 8 + n:pos + 12 + n])[0] == zlib.crc32(t + body)
        if t == b"IHDR":
            w, h, depth, ct = struct.unpack(">IIBB", body[:10])
            assert depth == 16 and ct == 0
        elif t == b"IDAT":
            idat += body
        pos += 12 + n
    raw = zlib.decompress(idat)
    rows = [raw[y * (2 * w + 1) + 1:(y + 1) * (2 * w + 1)] for y in range(h)]
    assert all(raw[y * (2 * w + 1)] == 0 for y in range(h))
    return np.frombuffer(b"".join(rows), ">u2").reshape(h, w).astype(np.uint16)


def test_save16bitpng_roundtrip(lib, tmp_path):
    a = np.random.default_rng(3).integers(0, 65536, (31, 64), dtype=np.uint16)
    fn = str(tmp_path / "o.png").encode()
    assert lib.pfd_save_png16(fn, a.ctypes.data_as(C.POINTER(C.c_uint16)), 64, 31) == 0
    np.testing.assert_array_equal(_read_png16(tmp_path / "o.png"), a)
    got = _load(lib, tmp_path / "o.png")  # and back through the loader
    np.testing.assert_array_equal(got[..., 0], a.astype(np.float32) / np.float32(65535.0))


@pytest.mark.parametrize("little", [True, False])
def test_pfm_endianness_and_cap(lib, tmp_path, little):
    """Depth.cpp:455-525: no flip, no normalisation: v<0 -> 0, then min(v/10, 10)."""
    v = np.random.default_rng(4).normal(3, 8, (6, 9)).astype(np.float32)
    hdr = b"Pf\n9 6\n" + (b"-1.0\n" if little else b"1.0\n")
    open(tmp_path / "d.pfm", "wb").write(hdr + v.astype("<f4" if little else ">f4").tobytes())
    got = _load(lib, tmp_path / "d.pfm")
    ref = np.minimum(np.maximum(v, 0) / np.float32(10.0), np.float32(10.0))
    np.testing.assert_array_equal(got[..., 0], ref)


def test_pgm_and_rejections(lib, tmp_path):
    """8-bit PGM samples as stored (stb does not rescale a maxval below 255); a PGM with maxval
    above 255 is refused, as stb_image v2.23 refuses it."""
    a = np.random.default_rng(5).integers(0, 201, (4, 5), dtype=np.uint8)
    open(tmp_path / "a.pgm", "wb").write(b"P5\n# c\n5 4\n200\n" + a.tobytes())
    got = _load(lib, tmp_path / "a.pgm")
    np.testing.assert_array_equal(got[..., 0], a.astype(np.float32) / np.float32(255.0))
    b = a.astype(np.uint16) * 20
    open(tmp_path / "b.pgm", "wb").write(b"P5\n5 4\n4095\n" + b.astype(">u2").tobytes())
    assert _load(lib, tmp_path / "b.pgm") is None
    open(tmp_path / "x.jpg", "wb").write(b"\xff\xd8\xff\xe0" + b"\0" * 64)
    assert _load(lib, tmp_path / "x.jpg") is None
    assert _load(lib, tmp_path / "missing.png") is None
    open(tmp_path / "t.png", "wb").write(open(tmp_path / "a.pgm", "rb").read()[:5])
    assert _load(lib, tmp_path / "t.png") is None


def test_cli_leres_layout_matches_python(lib):
    f = np.zeros(60, np.float32)
    r = np.zeros(60, np.float32)
    lib.pfd_leres_layout(f.ctypes.data_as(C.POINTER(C.c_float)),
                         r.ctypes.data_as(C.POINTER(C.c_float)))
    lay = PL.leres_layout()
    np.testing.assert_array_equal(f.reshape(15, 4), lay.fovs)
    np.testing.assert_array_equal(r.reshape(15, 4), lay.ranges)


def test_cli_binary_usage():
    import subprocess
    out = subprocess.run([BIN], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and "usage" in out.stdout
    out = subprocess.run([BIN, "0", "a"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 1 and "argc>=6" in out.stdout
    out = subprocess.run([BIN, "0", "a", "b", "c", "d", "--shard", "2/2"], capture_output=True,
                         text=True, timeout=60)
    assert out.returncode == 2 and "bad --shard" in out.stdout


@pytest.mark.parametrize("mode,sub,restart", [("L", None, 0), ("RGB", 0, 0), ("RGB", 2, 0),
                                              ("RGB", 1, 0), ("L", None, 4), ("RGB", 2, 3)])
def test_jpeg_decoder_vs_libjpeg(lib, tmp_path, mode, sub, restart):
    """The JPEG decoder behind the loaders (pf_jpeg.cpp) beside PIL's libjpeg, as a sanity bound
    on PIL-encoded files: gray, 4:4:4, 4:2:0, 4:2:2, restart intervals, odd sizes.  The decoder
    is bit-exact to the reference's stb_image (tests/test_codecs_stb.py); stb and libjpeg differ
    from each other by up to 2 levels without chroma subsampling (their integer IDCTs and
    fixed-point colour conversions); with subsampled chroma only the mean is bounded (0.3): the
    upsamplers differ (stb rounds +8/+2 where libjpeg alternates +8/+7) and at an odd width
    stb's 4:2:2 edge column can differ from libjpeg's by a hundred levels on sharp chroma, which
    the reference reproduces and so does this decoder (checked against stb itself)."""
    Image = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(6)
    h, w = 75, 101
    yy, xx = np.mgrid[0:h, 0:w]
    base = (np.sin(xx / 9.0) * 60 + np.cos(yy / 7.0) * 50 + 128)
    if mode == "L":
        a = np.clip(base + rng.normal(0, 4, (h, w)), 0, 255).astype(np.uint8)
    else:
        a = np.clip(np.stack([base, 255 - base, (xx * 2 + yy) % 256], -1) +
                    rng.normal(0, 4, (h, w, 3)), 0, 255).astype(np.uint8)
    im = Image.fromarray(a, mode)
    kw = {"quality": 92}
    if sub is not None:
        kw["subsampling"] = sub
    if restart:
        kw["restart_marker_blocks"] = restart
    fn = tmp_path / "t.jpg"
    try:
        im.save(fn, "JPEG", **kw)
    except TypeError:
        kw.pop("restart_marker_blocks", None)
        im.save(fn, "JPEG", **kw)
    ref = np.asarray(Image.open(fn).convert(mode)).astype(np.int32)
    got = _load(lib, fn, 0)
    assert got is not None
    got = np.rint(got * 255.0).astype(np.int32)
    if mode == "L":
        assert got.shape == (h, w, 1)
        got = got[..., 0]
    else:
        assert got.shape == (h, w, 3)
    d = np.abs(got - ref)
    assert (sub in (1, 2) or d.max() <= 2) and d.mean() < 0.3, (d.max(), d.mean())


def test_jpeg_progressive_decoded(lib, tmp_path):
    """Progressive JPEG loads (stb_image does), within the libjpeg bound above."""
    Image = pytest.importorskip("PIL.Image")
    yy, xx = np.mgrid[0:40, 0:52]
    a = np.clip(np.sin(xx / 6.0) * 80 + yy * 2 + 60, 0, 255).astype(np.uint8)
    Image.fromarray(a, "L").save(tmp_path / "p.jpg", "JPEG", progressive=True, quality=90)
    got = _load(lib, tmp_path / "p.jpg")
    assert got is not None and got.shape == (40, 52, 1)
    ref = np.asarray(Image.open(tmp_path / "p.jpg")).astype(np.int32)
    d = np.abs(np.rint(got[..., 0] * 255.0).astype(np.int32) - ref)
    assert d.max() <= 2 and d.mean() < 0.3


def test_image_decoders_fuzz_sanitized(tmp_path):
    """Mutated PNG / JPEG / PFM files through the loaders, built host-only with ASan + UBSan
    (tools/fuzz/fuzz_images.cpp): corrupt inputs must be rejected, never read out of bounds."""
    import shutil
    Image = pytest.importorskip("PIL.Image")
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    csrc = os.path.join(os.path.dirname(os.path.dirname(panofuse.LIB_PATH)), "csrc")
    exe = tmp_path / "fuzz"
    r = subprocess_run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                        "-fno-sanitize-recover=all", "-I", csrc,
                        os.path.join(root, "tools", "fuzz", "fuzz_images.cpp"),
                        os.path.join(csrc, "pf_image.cpp"), os.path.join(csrc, "pf_jpeg.cpp"),
                        "-lz", "-o", str(exe)])
    assert r.returncode == 0, r.stderr
    rng = np.random.default_rng(0)
    a = rng.integers(0, 255, (40, 57, 3), dtype=np.uint8)
    Image.fromarray(a).save(tmp_path / "a.jpg", quality=90, subsampling=2)
    Image.fromarray(a[..., 0]).save(tmp_path / "b.jpg", quality=90)
    Image.fromarray(a).save(tmp_path / "c.png")
    Image.fromarray(a[..., 0].astype(np.uint16) * 257).save(tmp_path / "d.png")
    (tmp_path / "e.pfm").write_bytes(b"Pf\n5 4\n-1.0\n" + np.ones((4, 5), np.float32).tobytes())
    seeds = [str(tmp_path / n) for n in ("a.jpg", "b.jpg", "c.png", "d.png", "e.pfm")]
    r = subprocess_run([str(exe), "600", str(tmp_path / "cur.bin")] + seeds, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "decoded" in r.stdout


def subprocess_run(cmd, timeout=300):
    import subprocess
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("mode,quality", [("RGB", 3072), ("L", 100), ("RGB", 95)])
def test_jpeg_writer_roundtrip(lib, tmp_path, mode, quality):
    """The tile writer of the RGB export (pfd_save_jpeg; the reference's stbi_write_jpg at
    quality width*3, clamped to 100, 4:4:4, Main.cpp:320, stb_image_write.h:1448-1451; its bytes
    are pinned to stb's in tests/test_codecs_stb.py): a baseline JFIF file, always three
    components as stb writes it, that libjpeg (PIL) reads as 4:4:4 with all-one quantisers at
    quality >= 100.  Bar: decoded by libjpeg and by the in-tree decoder, the error against the
    input is no worse than libjpeg's own encoder at the same quality and sampling (max + 1
    level, mean x 1.15); odd sizes exercise the edge blocks."""
    import io
    Image = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(3)
    h, w = 67, 93
    yy, xx = np.mgrid[0:h, 0:w]
    base = np.sin(xx / 7.0) * 70 + np.cos(yy / 5.0) * 40 + 128
    if mode == "L":
        a = np.clip(base + rng.normal(0, 3, (h, w)), 0, 255).astype(np.uint8)
        c = 1
    else:
        a = np.clip(np.stack([base, 255 - base, (xx * 3 + yy) % 256], -1) +
                    rng.normal(0, 3, (h, w, 3)), 0, 255).astype(np.uint8)
        c = 3
    fn = tmp_path / "w.jpg"
    arr = np.ascontiguousarray(a)
    assert lib.pfd_save_jpeg(str(fn).encode(), arr.ctypes.data_as(C.POINTER(C.c_uint8)), w, h,
                             c, quality, 0) == 0
    im = Image.open(fn)
    assert im.format == "JPEG" and im.size == (w, h) and im.mode == "RGB"
    if quality >= 100:
        assert all(v == 1 for t in im.quantization.values() for v in t)
    assert im.layer[0][1:3] == (1, 1) and im.layer[1][1:3] == (1, 1)  # 4:4:4
    # stb writes gray as Y with neutral chroma: compare on the gray level
    pix = np.asarray(im.convert("L") if c == 1 else im)
    buf = io.BytesIO()  # libjpeg's own encoder at the same settings, the yardstick
    Image.fromarray(a, mode).save(buf, "JPEG", quality=min(quality, 100), subsampling=0)
    buf.seek(0)
    e = np.abs(np.asarray(Image.open(buf)).astype(np.int32) - a.astype(np.int32))
    d = np.abs(pix.astype(np.int32) - a.astype(np.int32))
    assert d.max() <= e.max() + 1 and d.mean() <= 1.15 * e.mean() + 0.02, (d.max(), d.mean(),
                                                                            e.max(), e.mean())
    got = _load(lib, fn, 0)
    got = np.rint(got * 255.0).astype(np.int32)
    got = (got[..., 0] if c == 1 else got).reshape(a.shape)
    d = np.abs(got - a.astype(np.int32))
    assert d.max() <= e.max() + 1 and d.mean() <= 1.15 * e.mean() + 0.02, (d.max(), d.mean(),
                                                                            e.max(), e.mean())
