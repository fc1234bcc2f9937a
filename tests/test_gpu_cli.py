"""GPU end-to-end of the mode-0 command line (Main.cpp:331-687):
bin/panofuse_main reads the baseline, the 15 LeReS-layout tiles and the ground truth from
folders with the reference's naming conventions, fuses on the GPU through the DepthNamespace
facade, and writes <raw>.png (u16), <raw>.aligned.txt, .res.png and .giv.png.

Bars: the fused u16 PNG is bit-exact against the CPU oracle's MergeDepthMaps on the same
(u16-quantised) inputs; the metrics file agrees with the oracle's ErrorData/ErrorEmap within
the tolerances of tests/test_gpu_metrics.py (plus the file's 6-decimal printing).  The first
test's tiles are 16-bit PNGs (the MiDaS naming of Main.cpp:570-573); test_mode0_cli_jpeg_inputs
covers the reference's JPEG conventions with stb-decoded pixels as the oracle's inputs."""
import math
import os
import struct
import subprocess
import zlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import panofuse  # noqa: E402
import pf_layouts as PL  # noqa: E402
import pf_synth  # noqa: E402
import pyoracle as O  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(panofuse.LIB_PATH))
BIN = os.path.join(ROOT, "bin", "panofuse_main")
MYPI = 3.14159265359
ZR = PL.ZENITH_RANGE


def _png16_write(path, a):
    h, w = a.shape
    raw = b"".join(b"\0" + a[y].astype(">u2").tobytes() for y in range(h))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d))
    open(path, "wb").write(b"\x89PNG\r\n\x1a\n" +
                           chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 16, 0, 0, 0, 0)) +
                           chunk(b"IDAT", zlib.compress(raw, 1)) + chunk(b"IEND", b""))


def _png16_read(path):
    d = open(path, "rb").read()
    pos, idat = 8, b""
    while pos < len(d):
        n = struct.unpack(">I", d[pos:pos + 4])[0]
        t, body = d[pos + 4:pos + 8], d[pos + 8:pos + 8 + n]
        if t == b"IHDR":
            w, h = struct.unpack(">II", body[:8])
        elif t == b"IDAT":
            idat += body
        pos += 12 + n
    raw = zlib.decompress(idat)
    return np.frombuffer(b"".join(raw[y * (2 * w + 1) + 1:(y + 1) * (2 * w + 1)]
                                  for y in range(h)), ">u2").reshape(h, w).astype(np.uint16)


def _cround(x):  # C round(): half away from zero
    return int(math.copysign(math.floor(abs(x) + 0.5), x))


def _q16(a):
    return (np.clip(a, 0, 1) * 65535.0 + 0.5).astype(np.uint16)


def test_mode0_cli_end_to_end(tmp_path):
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a host without a GPU")
    d = {k: tmp_path / k for k in ("rgb", "gt", "base", "result_hohonet", "tiles")}
    for p in d.values():
        p.mkdir()
    lay = PL.leres_layout(512, 494)
    tiles_o, total = O.make_tiles(lay)
    expected = {}
    for i, raw in enumerate(["scene01_rgb", "scene02_rgb"]):
        (d["rgb"] / (raw + ".jpg")).write_bytes(b"\xff\xd8")  # only the name is used
        seeds = pf_synth.seeds_for(1, 20261015 + 31 * i)
        gt = _q16(pf_synth.scene_depth(seeds, 2048, 1024)[0].numpy())
        base = _q16(pf_synth.baseline_emap(seeds, 512, 256)[0].numpy())
        _png16_write(d["gt"] / (raw.replace("_rgb", "_depth") + ".png"), gt)
        _png16_write(d["base"] / (raw + ".depth.png"), base)  # hohonet naming (Main.cpp:512-516)
        gt_f = gt.astype(np.float32) / np.float32(65535.0)
        resp = pf_synth.responses(seeds, lay.ntiles)
        tdata = O.warp_depth(gt_f, tiles_o, total, O.responses(resp))
        tq = _q16(tdata)
        off = 0
        for t in range(lay.ntiles):
            f = [_cround(float(v) / MYPI * 180.0) for v in lay.fovs[t]]
            name = f"{raw}.{f[0]}_{f[1]}_{f[2]}_{f[3]}.png"
            n = 512 * 494
            _png16_write(d["tiles"] / name, tq[off:off + n].reshape(494, 512))
            off += n
        base_f = base.astype(np.float32) / np.float32(65535.0)
        out, _ = O.merge(base_f, tiles_o, tq.astype(np.float32) / np.float32(65535.0), 2048, ZR)
        expected[raw] = (out, gt_f, base_f)

    cmd = [BIN, "0", str(d["rgb"]), str(d["gt"]), str(d["base"]), str(d["result_hohonet"]),
           "--tiles", str(d["tiles"])]
    # one process per shard (as one per GPU): shard 0/2 takes scene01 (metrics in the default
    # order: the reference's float sums), 1/2 scene02 (--metrics-order tree: the fp64 tree)
    for k, raw in enumerate(sorted(expected)):
        order = ["--metrics-order", "tree"] if k == 1 else []
        r = subprocess.run(cmd + ["--shard", f"{k}/2"] + order, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "#RGB_filenames:1" in r.stdout
        assert (d["result_hohonet"] / (raw + ".png")).exists()
    for raw, (out, gt_f, base_f) in expected.items():
        got = _png16_read(d["result_hohonet"] / (raw + ".png"))
        assert got.shape == (1024, 2048)
        bad = int((got != out).sum())
        assert bad == 0, f"{raw}: {bad} pixels differ from the oracle"
        for suffix in (".png.res.png", ".png.giv.png"):
            assert (d["result_hohonet"] / (raw + suffix)).exists()
        txt = (d["result_hohonet"] / (raw + ".aligned.txt")).read_text()
        vals = dict(line.split(": ") for line in txt.strip().splitlines())
        ref_r = O.error_metrics(gt_f, out, ZR, 1, True)
        ref_g = O.error_metrics(gt_f, base_f, ZR, 1, True)
        seq = raw == sorted(expected)[0]
        for key, ref in (("result", ref_r), ("given", ref_g)):
            for m in ("mse", "mae", "mre", "mselog"):
                # sequential: the oracle's float sums up to the file's "%f" printing (and
                # mselog's 1e-5, test_gpu_metrics.py); tree: within the drift of those sums
                got = float(vals[f"{m}_{key}"])
                if seq:
                    tol = 5.01e-7 + (1e-5 * abs(ref[m]) if m == "mselog" else 0.0)
                    assert abs(got - ref[m]) <= tol, (raw, key, m, got, ref[m])
                else:
                    assert got == pytest.approx(ref[m], rel=1e-2, abs=1e-6)
            for m in ("delta1", "delta2", "delta3"):
                assert float(vals[f"{m}_{key}"]) == pytest.approx(ref[m], abs=1e-6)
    # second run: every output exists -> skipped (Main.cpp:552-561)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.count("skip!") == 2


def _png8_read(path):
    d = open(path, "rb").read()
    pos, idat = 8, b""
    while pos < len(d):
        n = struct.unpack(">I", d[pos:pos + 4])[0]
        t, body = d[pos + 4:pos + 8], d[pos + 8:pos + 8 + n]
        if t == b"IHDR":
            w, h, depth, ct = struct.unpack(">IIBB", body[:10])
            assert depth == 8 and ct == 2
        elif t == b"IDAT":
            idat += body
        pos += 12 + n
    raw = zlib.decompress(idat)
    return np.frombuffer(b"".join(raw[y * (3 * w + 1) + 1:(y + 1) * (3 * w + 1)]
                                  for y in range(h)), np.uint8).reshape(h, w, 3)


def _png8_write_rgb(path, a):
    h, w, _ = a.shape
    raw = b"".join(b"\0" + a[y].tobytes() for y in range(h))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d))
    open(path, "wb").write(b"\x89PNG\r\n\x1a\n" +
                           chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)) +
                           chunk(b"IDAT", zlib.compress(raw, 1)) + chunk(b"IEND", b""))


def test_export_rgb_tiles(tmp_path):
    """`panofuse_main export`: the tile render of mode 0 (SaveCubeMap, Main.cpp:242-326) for
    the LeReS layout at 1024 x 988 px, written as JPEG at quality 100 / 4:4:4 (Main.cpp:320)
    and decoded here by libjpeg (PIL), against the oracle's restatement of the GL camera: the
    warp itself is bit-exact (test_gpu_parity.py::test_warp_rgb_bit_exact), so what remains is
    the JPEG round trip's bar (tests/test_io.py), i.e. within 4 levels, mean under 0.5.  OpenGL
    rasterisation parity is unpinned.  Every file must also equal, byte for byte, the
    reference's own stbi_write_jpg of the oracle's tile at the reference's quality argument:
    tests/golden/export_rgb_stb.json holds those files' SHA-256, recorded in the build container
    from the stb build of /root/reference (tools/make_stb_golden.py export), so no
    reference-built code runs here."""
    import hashlib
    import json

    import codec_cases as CC
    Image = pytest.importorskip("PIL.Image")
    golden = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                         "export_rgb_stb.json")))
    (tmp_path / "rgb").mkdir()
    pano = CC.export_pano()
    _png8_write_rgb(tmp_path / "rgb" / "room7.png", pano)
    r = subprocess.run([BIN, "export", str(tmp_path / "rgb"), str(tmp_path / "tiles")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    lay = PL.leres_layout(1024, 988)
    assert len(golden["tiles"]) == lay.ntiles and golden["quality"] == 1024 * 3
    tiles_o, _ = O.make_tiles(lay)
    ref = O.warp_rgb(pano, tiles_o)
    off = 0
    for t in range(lay.ntiles):
        f = [_cround(float(v) / MYPI * 180.0) for v in lay.fovs[t]]
        fn = tmp_path / "tiles" / f"room7.{f[0]}_{f[1]}_{f[2]}_{f[3]}.jpg"
        assert hashlib.sha256(fn.read_bytes()).hexdigest() == golden["tiles"][t], t
        im = Image.open(fn)
        assert im.format == "JPEG" and im.mode == "RGB"
        got = np.asarray(im)
        assert got.shape == (988, 1024, 3)
        n = 988 * 1024 * 3
        d = np.abs(got.reshape(-1).astype(np.int32) - ref[off:off + n].astype(np.int32))
        off += n
        assert d.max() <= 4 and d.mean() < 0.5, (t, d.max(), d.mean())


def test_mode0_cli_jpeg_inputs(tmp_path):
    """The reference's own file conventions: LeReS tiles as 8-bit gray JPEG in test_images
    naming (<raw>.<a0>_<a1>_<z0>_<z1>.jpg, Main.cpp:576-578) and a bifuse baseline <raw>.jpg
    (Main.cpp:499).  The oracle is run on the pixels the reference's stb_image decodes from
    those files: tests/golden/cli_jpeg_stb.json (tools/make_stb_golden.py, from the stb build of
    /root/reference) records each file's SHA-256 and the SHA-256 of stb's decode; the files
    generated here must hash the same, and the facade's decoder must reproduce stb's hashes, so
    the oracle's inputs below are stb's pixels.  The CLI's fused u16 output is then bit-exact
    against the oracle."""
    import ctypes as C
    import hashlib
    import json

    import codec_cases as CC
    pytest.importorskip("PIL.Image")
    L = C.CDLL(os.path.join(os.path.dirname(panofuse.LIB_PATH), "libpanofuse_depth.so"))
    ip = C.POINTER(C.c_int)
    L.pfd_decode_image.argtypes = [C.c_char_p, C.c_void_p, C.c_longlong, ip, ip, ip, ip]
    golden = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                         "cli_jpeg_stb.json")))

    def stb_pixels(fn):
        rec = golden[fn.name]
        assert hashlib.sha256(fn.read_bytes()).hexdigest() == rec["file_sha256"], fn.name
        w, h, c, s16 = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        buf = np.zeros(1 << 22, np.uint8)
        assert L.pfd_decode_image(str(fn).encode(), buf.ctypes.data, buf.size, C.byref(w),
                                  C.byref(h), C.byref(c), C.byref(s16)) == 0
        px = buf[:w.value * h.value * c.value].reshape(h.value, w.value, c.value)
        assert list(px.shape) == rec["stb_shape"]
        assert hashlib.sha256(px.tobytes()).hexdigest() == rec["stb_px_sha256"], fn.name
        return px.astype(np.float32) / np.float32(255.0)  # Depth.cpp:96-98

    d = {k: tmp_path / k for k in ("rgb", "gt", "base", "result", "test_images")}
    for p in d.values():
        p.mkdir()
    raw, names, base_fn, gt = CC.cli_jpeg_inputs(d)
    (d["rgb"] / (raw + ".png")).write_bytes(b"\x89PNG")
    _png16_write(d["gt"] / "room_depth.png", gt)
    lay = PL.leres_layout(512, 494)
    tiles_o, _ = O.make_tiles(lay)
    dec = np.concatenate([stb_pixels(fn)[..., 0].reshape(-1) for fn in names])
    base_f = stb_pixels(base_fn)[..., 0]
    ref, _ = O.merge(base_f, tiles_o, dec, 2048, ZR)
    cmd = [BIN, "0", str(d["rgb"]), str(d["gt"]), str(d["base"]), str(d["result"]), "--tiles",
           str(d["test_images"])]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    got = _png16_read(d["result"] / (raw + ".png"))
    assert int((got != ref).sum()) == 0
