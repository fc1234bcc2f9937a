"""The image codecs either side of the path held to the reference's own: stb_image v2.23 and
stb_image_write v1.15.

The reference decodes every map it loads with stbi_load / stbi_load_16 (req_comp 0,
Depth.cpp:45-109, 277-355) -- its depth-net tiles are JPEG (Main.cpp:576-578) -- and writes the
RGB tiles with stbi_write_jpg (Main.cpp:319-320).  The bar is bit-exact: same channel count,
same samples, same bytes.

* With the reference's stb compiled from /root/reference (oracle/_ref/libstbref.so, built by
  oracle/Makefile; it travels with the snapshot): PIL-encoded JPEGs (gray / RGB / CMYK, 4:4:4 /
  4:2:2 / 4:2:0, baseline / progressive, restart intervals, optimised tables, 1-pixel and odd
  sizes) and PNGs written here (every colour type and depth, Adam7, palette / colour-key tRNS)
  decoded by both; JPEG writes at qualities 0..3072, 1..4 channels, flipped or not.
* Everywhere, with no stb present: tests/golden/stb_codecs.npz (tools/make_stb_golden.py) holds
  such files with the pixels stb decoded from them and the bytes stb wrote -- the same checks
  against the recorded answers.
No device calls.
"""
import ctypes as C
import os

import numpy as np
import pytest

import codec_cases as CC
import panofuse
import pystb

LIB = os.path.join(os.path.dirname(panofuse.LIB_PATH), "libpanofuse_depth.so")
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "stb_codecs.npz")
need_stb = pytest.mark.skipif(not pystb.available(), reason="no oracle/_ref/libstbref.so")


@pytest.fixture(scope="module")
def lib():
    L = C.CDLL(LIB)
    ip = C.POINTER(C.c_int)
    L.pfd_decode_image.argtypes = [C.c_char_p, C.c_void_p, C.c_longlong, ip, ip, ip, ip]
    L.pfd_is_16_bit.argtypes = [C.c_char_p]
    L.pfd_save_jpeg.argtypes = [C.c_char_p, C.POINTER(C.c_uint8), C.c_int, C.c_int, C.c_int,
                                C.c_int, C.c_int]
    return L


def decode(lib, fn):
    """the facade's decoder: [h][w][c] uint8 / uint16 as loaded, or None"""
    w, h, c, s = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    buf = np.zeros(1 << 24, np.uint8)
    rc = lib.pfd_decode_image(str(fn).encode(), buf.ctypes.data, buf.size, C.byref(w),
                              C.byref(h), C.byref(c), C.byref(s))
    if rc:
        return None
    n = w.value * h.value * c.value
    a = buf[:n * (2 if s.value else 1)]
    a = a.view(np.uint16) if s.value else a
    return a.reshape(h.value, w.value, c.value).copy()


def encode(lib, fn, px, q, flip):
    px = np.ascontiguousarray(px, np.uint8)
    h, w, c = px.shape
    assert lib.pfd_save_jpeg(str(fn).encode(), px.ctypes.data_as(C.POINTER(C.c_uint8)), w, h, c,
                             q, int(flip)) == 0
    return open(fn, "rb").read()


def _write(tmp_path, name, data):
    fn = tmp_path / name.replace("/", "_")
    fn.write_bytes(data)
    return fn


JPEGS = CC.jpeg_cases(seed=11, n=32)
PNGS = CC.png_cases(seed=5)


@need_stb
@pytest.mark.parametrize("name,data", JPEGS, ids=[c[0] for c in JPEGS])
def test_jpeg_decode_matches_stb(lib, tmp_path, name, data):
    fn = _write(tmp_path, name + ".jpg", data)
    ref = pystb.load(fn, want16=False)
    got = decode(lib, fn)
    assert ref is not None and got is not None
    assert got.shape == ref.shape and got.dtype == ref.dtype
    assert np.array_equal(got, ref), int((got != ref).sum())


@need_stb
@pytest.mark.parametrize("name,data", PNGS, ids=[c[0] for c in PNGS])
def test_png_decode_matches_stb(lib, tmp_path, name, data):
    fn = _write(tmp_path, name + ".png", data)
    is16 = pystb.is_16_bit(fn)
    assert bool(lib.pfd_is_16_bit(str(fn).encode())) == is16
    ref = pystb.load(fn)  # stbi_load_16 when stbi_is_16_bit, as the reference's Load decides
    got = decode(lib, fn)
    assert ref is not None and got is not None
    assert got.shape == ref.shape and got.dtype == ref.dtype, (got.shape, ref.shape, got.dtype)
    assert np.array_equal(got, ref)


@need_stb
@pytest.mark.parametrize("name,px,q,flip", CC.writer_cases(seed=2),
                         ids=[c[0] for c in CC.writer_cases(seed=2)])
def test_jpeg_writer_matches_stb_bytes(lib, tmp_path, name, px, q, flip):
    pystb.write_jpg(tmp_path / "ref.jpg", px, q, flip)
    ref = (tmp_path / "ref.jpg").read_bytes()
    got = encode(lib, tmp_path / "got.jpg", px, q, flip)
    assert got == ref, (len(got), len(ref))


@need_stb
def test_rejections_match_stb(lib, tmp_path):
    """Files stb refuses are refused: a 16-bit PGM (stb 2.23's PNM reader is 8-bit only), an
    arithmetic-coded / lossless SOF, a JPEG without EOI, a PNG with an unknown critical chunk."""
    import struct
    import zlib
    a = np.arange(20, dtype=np.uint16).reshape(4, 5) * 200
    cases = {"p16.pgm": b"P5\n5 4\n4095\n" + a.astype(">u2").tobytes(),
             "sof3.jpg": bytes.fromhex("ffd8ffc3000b080001000101011100ffd9"),
             "noeoi.jpg": JPEGS[4][1][:-2]}
    png = CC.png_bytes(np.zeros((2, 2, 1), int), 8, 0)
    bad = struct.pack(">I", 0) + b"ABCD" + struct.pack(">I", zlib.crc32(b"ABCD"))
    cases["crit.png"] = png[:33] + bad + png[33:]
    for n, d in cases.items():
        fn = _write(tmp_path, n, d)
        assert pystb.load(fn, want16=False) is None, n
        assert decode(lib, fn) is None, n


def test_golden_decodes(lib, tmp_path):
    """The recorded stb decodes (tests/golden/stb_codecs.npz) reproduced bit for bit."""
    g = np.load(GOLDEN, allow_pickle=False)
    names = sorted({k[:-5] for k in g.files if k.endswith("_file")})
    assert len(names) >= 40
    for n in names:
        fn = _write(tmp_path, n + (".jpg" if n.startswith("jpg") else ".png"), g[n + "_file"].tobytes())
        got = decode(lib, fn)
        ref = g[n + "_px"]
        assert got is not None, n
        assert got.shape == ref.shape and got.dtype == ref.dtype, n
        assert np.array_equal(got, ref), n


def test_golden_jpeg_writes(lib, tmp_path):
    """The recorded stbi_write_jpg outputs (tests/golden/stb_codecs.npz) reproduced byte for byte."""
    g = np.load(GOLDEN, allow_pickle=False)
    names = sorted({k[:-3] for k in g.files if k.startswith("w") and k.endswith("_in")})
    assert len(names) >= 6
    for n in names:
        q, flip = (int(v) for v in g[n + "_meta"])
        assert encode(lib, tmp_path / "o.jpg", g[n + "_in"], q, flip) == g[n + "_out"].tobytes(), n
