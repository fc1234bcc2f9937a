"""Image files for the codec parity tests (tests/test_codecs_stb.py, tools/make_stb_golden.py):
JPEGs from PIL's libjpeg encoder with the options the reference's inputs come with (gray / RGB /
CMYK, 4:4:4 / 4:2:2 / 4:2:0, baseline / progressive, restart intervals, optimised Huffman
tables, odd and one-pixel sizes) and PNGs written here (every colour type and bit depth, all
five filters, Adam7 interlacing, palette and colour-key tRNS).  Deterministic for a seed."""
import struct
import zlib

import numpy as np


def _chunk(t, d):
    return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return a if pa <= pb and pa <= pc else (b if pb <= pc else c)


def _filter(ft, row, prev, bpp):
    out = bytearray(len(row))
    for i in range(len(row)):
        a = row[i - bpp] if i >= bpp else 0
        b = prev[i] if prev is not None else 0
        c = prev[i - bpp] if (prev is not None and i >= bpp) else 0
        out[i] = (row[i] - [0, a, b, (a + b) >> 1, _paeth(a, b, c)][ft]) & 0xFF
    return bytes(out)


def _pack_row(samples, depth):
    """samples: 1-D int array of one row (all channels interleaved)"""
    if depth == 16:
        return samples.astype(">u2").tobytes()
    if depth == 8:
        return samples.astype(np.uint8).tobytes()
    per = 8 // depth
    out = bytearray((len(samples) + per - 1) // per)
    for i, v in enumerate(samples):
        out[i // per] |= int(v) << (8 - depth - (i % per) * depth)
    return bytes(out)


ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2),
         (0, 1, 1, 2)]


def png_bytes(img, depth, ctype, interlace=False, plte=None, trns=None, seed=0):
    """img: [h][w][nc] ints (palette: indices).  Filter types cycle per row."""
    h, w = img.shape[:2]
    nc = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    bpp = max(1, nc * depth // 8)
    raw = b""
    passes = ADAM7 if interlace else [(0, 0, 1, 1)]
    ft = seed % 5
    for x0, y0, dx, dy in passes:
        sub = img[y0::dy, x0::dx]
        if sub.size == 0:
            continue
        prev = None
        for y in range(sub.shape[0]):
            row = _pack_row(sub[y].reshape(-1), depth)
            raw += bytes([ft]) + _filter(ft, row, prev, bpp)
            prev = row
            ft = (ft + 1) % 5
    data = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0,
                                                               0, int(interlace)))
    if plte is not None:
        data += _chunk(b"PLTE", plte)
    if trns is not None:
        data += _chunk(b"tRNS", trns)
    z = zlib.compress(raw)
    return data + _chunk(b"IDAT", z[:len(z) // 2]) + _chunk(b"IDAT", z[len(z) // 2:]) + \
        _chunk(b"IEND", b"")


def png_cases(seed=0, n=None):
    """[(name, bytes)] covering colour type x depth x interlace x tRNS."""
    rng = np.random.default_rng(seed)
    cases = []
    combos = [(0, d) for d in (1, 2, 4, 8, 16)] + [(2, 8), (2, 16), (3, 1), (3, 2), (3, 4),
                                                  (3, 8), (4, 8), (4, 16), (6, 8), (6, 16)]
    k = 0
    for ctype, depth in combos:
        for interlace in (False, True):
            for key in (False, True):
                if key and ctype in (4, 6):
                    continue
                h, w = (int(v) for v in rng.integers(1, 23, 2))
                nc = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
                plte = trns = None
                if ctype == 3:
                    npal = int(rng.integers(1, 1 << depth)) + 1 if depth < 8 else 200
                    npal = min(npal, 1 << depth)
                    img = rng.integers(0, npal, (h, w, 1))
                    plte = rng.integers(0, 256, 3 * npal, dtype=np.uint8).tobytes()
                    if key:
                        trns = rng.integers(0, 256, int(rng.integers(1, npal + 1)),
                                            dtype=np.uint8).tobytes()
                else:
                    img = rng.integers(0, 1 << depth, (h, w, nc))
                    if key:  # a key that some pixels match
                        kv = img[0, 0].copy()
                        img[h // 2:, : w // 2] = kv
                        trns = b"".join(struct.pack(">H", int(v)) for v in kv)
                cases.append((f"png_c{ctype}_d{depth}_i{int(interlace)}_k{int(key)}",
                              png_bytes(img, depth, ctype, interlace, plte, trns, seed=k)))
                k += 1
    return cases if n is None else cases[:n]


def jpeg_cases(seed=0, n=24):
    """[(name, bytes)] from PIL's encoder."""
    import io

    from PIL import Image
    rng = np.random.default_rng(seed)
    cases = []
    sizes = [(1, 1), (1, 17), (9, 1), (8, 8), (16, 16), (17, 33), (75, 101), (33, 7)]
    for i in range(n):
        mode = ["L", "RGB", "RGB", "CMYK"][i % 4]
        h, w = sizes[i % len(sizes)] if i < len(sizes) else tuple(int(v) for v in rng.integers(2, 90, 2))
        ch = {"L": 1, "RGB": 3, "CMYK": 4}[mode]
        yy, xx = np.mgrid[0:h, 0:w]
        base = np.sin(xx / 5.0) * 60 + np.cos(yy / 4.0) * 50 + 128
        a = np.clip(np.stack([base + 37 * k for k in range(ch)], -1) +
                    rng.normal(0, 15, (h, w, ch)), 0, 255).astype(np.uint8)
        kw = {"quality": int(rng.integers(20, 101))}
        if ch > 1:
            kw["subsampling"] = int(i // 4 % 3)
        if i % 3 == 1:
            kw["progressive"] = True
        if i % 5 == 2:
            kw["restart_marker_blocks"] = int(rng.integers(1, 4))
        if i % 7 == 3:
            kw["optimize"] = True
        buf = io.BytesIO()
        Image.fromarray(a[..., 0] if ch == 1 else a, mode).save(buf, "JPEG", **kw)
        tag = "_".join(f"{k}{int(v) if not isinstance(v, bool) else int(v)}" for k, v in kw.items())
        cases.append((f"jpg_{mode}_{h}x{w}_{tag}", buf.getvalue()))
    return cases


def writer_cases(seed=0):
    """[(name, pixels [h][w][c] uint8, quality, flip)] for stbi_write_jpg parity."""
    rng = np.random.default_rng(seed)
    out = []
    for i, (q, c, flip) in enumerate([(3072, 3, True), (100, 1, False), (95, 3, False),
                                      (90, 3, True), (50, 4, False), (10, 2, True),
                                      (0, 3, False), (1, 3, False)]):
        h, w = (int(v) for v in rng.integers(1, 41, 2))
        yy, xx = np.mgrid[0:h, 0:w]
        base = np.sin(xx / 4.0) * 70 + np.cos(yy / 6.0) * 40 + 128
        px = np.clip(np.stack([base + 50 * k for k in range(c)], -1) + rng.normal(0, 9, (h, w, c)),
                     0, 255).astype(np.uint8)
        out.append((f"w{i}_q{q}_c{c}_f{int(flip)}", px, q, flip))
    return out


def cli_jpeg_inputs(d, quality=95):
    """The reference's mode-0 file conventions with JPEG inputs (tests/test_gpu_cli.py
    test_mode0_cli_jpeg_inputs): LeReS-layout tiles as 8-bit gray JPEG in test_images naming
    (<raw>.<a0>_<a1>_<z0>_<z1>.jpg, Main.cpp:576-578), a bifuse baseline <raw>.jpg
    (Main.cpp:499) and a 16-bit ground truth, written under the dict of folders d.  Returns
    (raw, tile file names in layout order, baseline file name, gt u16 array).  CPU only."""
    import math

    from PIL import Image

    import pf_layouts as PL
    import pf_synth
    import pyoracle as O

    def cround(x):
        return int(math.copysign(math.floor(abs(x) + 0.5), x))

    lay = PL.leres_layout(512, 494)
    tiles_o, total = O.make_tiles(lay)
    raw = "room_rgb"
    seeds = pf_synth.seeds_for(1, 20261015 + 555)
    gt = (np.clip(pf_synth.scene_depth(seeds, 2048, 1024)[0].numpy(), 0, 1) * 65535.0 + 0.5
          ).astype(np.uint16)
    base8 = (np.clip(pf_synth.baseline_emap(seeds, 512, 256)[0].numpy(), 0, 1) * 255 + 0.5
             ).astype(np.uint8)
    base_fn = d["base"] / (raw + ".jpg")
    Image.fromarray(base8, "L").save(base_fn, "JPEG", quality=quality)
    gt_f = gt.astype(np.float32) / np.float32(65535.0)
    tdata = O.warp_depth(gt_f, tiles_o, total, O.responses(pf_synth.responses(seeds, lay.ntiles)))
    t8 = (np.clip(tdata, 0, 1) * 255 + 0.5).astype(np.uint8)
    names, off = [], 0
    for t in range(lay.ntiles):
        f = [cround(float(v) / 3.14159265359 * 180.0) for v in lay.fovs[t]]
        fn = d["test_images"] / f"{raw}.{f[0]}_{f[1]}_{f[2]}_{f[3]}.jpg"
        Image.fromarray(t8[off:off + 512 * 494].reshape(494, 512), "L").save(fn, "JPEG",
                                                                              quality=quality)
        names.append(fn)
        off += 512 * 494
    return raw, names, base_fn, gt


def export_pano(h=512, w=1024, seed=9):
    """The RGB panorama of tests/test_gpu_cli.py::test_export_rgb_tiles (and of its stb fixture,
    tests/golden/export_rgb_stb.json): a horizontal and a vertical ramp plus a noise channel."""
    rs = np.random.RandomState(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    return np.stack([(xx * 255 // (w - 1)), (yy * 255 // (h - 1)),
                     rs.randint(0, 256, size=(h, w))], -1).astype(np.uint8)
