"""Regenerate tests/golden/stb_codecs.npz: image files (tests/codec_cases.py) with the pixels the
reference's stb_image decodes from them, and pixel arrays with the bytes its stbi_write_jpg
writes -- answers recorded from the reference's own codecs (oracle/_ref/libstbref.so, compiled
from /root/reference by oracle/Makefile), for the stb-free checks in tests/test_codecs_stb.py.

Usage (build container, after `make -C oracle`): python tools/make_stb_golden.py"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import codec_cases as CC  # noqa: E402
import pystb  # noqa: E402


def main():
    if not pystb.available():
        sys.exit("oracle/_ref/libstbref.so not built (needs /root/reference)")
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for name, data in CC.jpeg_cases(seed=101, n=24) + CC.png_cases(seed=7):
            fn = os.path.join(d, "f")
            open(fn, "wb").write(data)
            px = pystb.load(fn)
            assert px is not None, name
            out[name + "_file"] = np.frombuffer(data, np.uint8)
            out[name + "_px"] = px
        for name, px, q, flip in CC.writer_cases(seed=9):
            fn = os.path.join(d, "w.jpg")
            assert pystb.write_jpg(fn, px, q, flip)
            out[name + "_in"] = px
            out[name + "_meta"] = np.array([q, int(flip)], np.int32)
            out[name + "_out"] = np.frombuffer(open(fn, "rb").read(), np.uint8)
    dst = os.path.join(ROOT, "tests", "golden", "stb_codecs.npz")
    np.savez_compressed(dst, **out)
    print(dst, os.path.getsize(dst), "bytes,", len(out), "arrays")
    cli_fixture()
    export_fixture()


def export_fixture():
    """SHA-256 of the reference's own stbi_write_jpg (quality argument = the row stride,
    Main.cpp:320) applied to the oracle's RGB tiles of tests/test_gpu_cli.py::
    test_export_rgb_tiles (LeReS layout at 1024 x 988, panorama codec_cases.export_pano()):
    tests/golden/export_rgb_stb.json.  The GPU test compares its exported files with these
    hashes, so the reference-built codec never has to travel to the GPU box."""
    import hashlib
    import json
    sys.path.insert(0, os.path.join(ROOT, "wacv2023-high-resolution-depth-estimation-for-"
                                          "panoramas-through-perspective-map-registrations_amd"))
    import pf_layouts as PL
    import pyoracle as O
    lay = PL.leres_layout(1024, 988)
    tiles_o, _ = O.make_tiles(lay)
    ref = O.warp_rgb(CC.export_pano(), tiles_o)
    n = 988 * 1024 * 3
    rec = {"layout": "LeReS 1024x988", "quality": 1024 * 3, "tiles": []}
    with tempfile.TemporaryDirectory() as d:
        for t in range(lay.ntiles):
            fn = os.path.join(d, "t.jpg")
            assert pystb.write_jpg(fn, ref[t * n:(t + 1) * n].reshape(988, 1024, 3), 1024 * 3)
            rec["tiles"].append(hashlib.sha256(open(fn, "rb").read()).hexdigest())
    dst = os.path.join(ROOT, "tests", "golden", "export_rgb_stb.json")
    json.dump(rec, open(dst, "w"), indent=1)
    print(dst, len(rec["tiles"]), "tiles")


def cli_fixture():
    """SHA-256 of the JPEG inputs of tests/test_gpu_cli.py::test_mode0_cli_jpeg_inputs and of
    the pixels stb decodes from them (tests/golden/cli_jpeg_stb.json)."""
    import hashlib
    import json
    import pathlib
    sys.path.insert(0, os.path.join(ROOT, "wacv2023-high-resolution-depth-estimation-for-"
                                          "panoramas-through-perspective-map-registrations_amd"))
    rec = {}
    with tempfile.TemporaryDirectory() as d:
        dirs = {k: pathlib.Path(d) / k for k in ("base", "test_images")}
        for p in dirs.values():
            p.mkdir()
        raw, names, base_fn, _ = CC.cli_jpeg_inputs(dirs)
        for fn in [base_fn] + names:
            px = pystb.load(fn, want16=False)
            rec[fn.name] = {"file_sha256": hashlib.sha256(fn.read_bytes()).hexdigest(),
                            "stb_shape": list(px.shape),
                            "stb_px_sha256": hashlib.sha256(px.tobytes()).hexdigest()}
    dst = os.path.join(ROOT, "tests", "golden", "cli_jpeg_stb.json")
    json.dump(rec, open(dst, "w"), indent=1, sort_keys=True)
    print(dst, len(rec), "files")


if __name__ == "__main__":
    if sys.argv[1:] == ["export"]:  # only the export-tile hashes
        if not pystb.available():
            sys.exit("oracle/_ref/libstbref.so not built (needs /root/reference)")
        export_fixture()
    else:
        main()
