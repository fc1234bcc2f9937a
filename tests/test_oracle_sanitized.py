"""The oracle under AddressSanitizer + UBSan ("ASan/UBSan on the CPU
restatement") -- CPU only.

tests/cpp/oracle_asan.c links oracle/pf_oracle.c and pf_oracle_lm.c built with
-fsanitize=address,undefined -fno-sanitize-recover=all and runs the E->P depth warp, the
MergeDepthMaps core (registration + 3-level fusion + u16), the RGB warp and SolveDepthBySmoothing
on the C1 layout.  Any out-of-bounds access or undefined behaviour aborts it.  Its outputs must
equal the unsanitized oracle's (tests use liboracle.so through pyoracle), so the sanitized run
exercised the same code paths, bit for bit."""
import ctypes as C
import os
import shutil
import subprocess

import numpy as np
import pytest

import pf_layouts as PL
import pf_synth
import pyoracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_under_asan_ubsan(tmp_path):
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    exe = tmp_path / "oracle_asan"
    r = subprocess.run(["gcc", "-std=gnu11", "-O1", "-g", "-fopenmp", "-ffp-contract=off",
                        "-fno-fast-math", "-fsanitize=address,undefined",
                        "-fno-sanitize-recover=all", "-I", os.path.join(ROOT, "oracle"),
                        os.path.join(ROOT, "tests", "cpp", "oracle_asan.c"),
                        os.path.join(ROOT, "oracle", "pf_oracle.c"),
                        os.path.join(ROOT, "oracle", "pf_oracle_lm.c"), "-lm", "-o", str(exe)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]

    lay = PL.config_layout("C1")
    zr = PL.ZENITH_RANGE
    tiles, total = O.make_tiles(lay)
    pw, ph, ew, eh, out_w = 512, 256, 128, 64, 512
    seeds = pf_synth.seeds_for(1, 20261017)
    pano = pf_synth.scene_depth(seeds, pw, ph, "cpu").numpy().reshape(ph, pw).astype(np.float32)
    emap = pf_synth.baseline_emap(seeds, ew, eh, "cpu").numpy().reshape(eh, ew).astype(np.float32)
    rp = pf_synth.responses(seeds, lay.ntiles)
    resp = O.responses(rp)
    rng = np.random.default_rng(5)
    rgb = rng.integers(0, 256, (ph, pw, 3), dtype=np.uint8)

    d = tmp_path / "case"
    d.mkdir()
    (d / "case.bin").write_bytes(np.array([lay.ntiles, total, pw, ph, ew, eh, out_w], np.int32)
                                 .tobytes() + np.array(zr, np.float32).tobytes())
    (d / "tiles.bin").write_bytes(bytes(tiles))
    (d / "resp.bin").write_bytes(bytes(resp))
    (d / "pano.f32").write_bytes(pano.tobytes())
    (d / "emap.f32").write_bytes(emap.tobytes())
    (d / "rgb.u8").write_bytes(rgb.tobytes())
    env = dict(os.environ, OMP_NUM_THREADS="2",
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1")
    r = subprocess.run([str(exe), str(d)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "oracle_asan ok" in r.stdout

    # the unsanitized oracle on the same inputs
    tile_data = O.warp_depth(pano, tiles, total, resp)
    warped = tile_data.copy()
    ref_out, ref_abcd = O.merge(emap, tiles, tile_data, out_w, zr)
    got = np.frombuffer((d / "out.u16").read_bytes(), np.uint16).reshape(out_w // 2, out_w)
    assert np.array_equal(got, ref_out)
    abcd = np.frombuffer((d / "abcd.f32").read_bytes(), np.float32).reshape(-1, 4)
    assert np.array_equal(abcd.view(np.uint32), ref_abcd.view(np.uint32))
    assert np.array_equal(np.frombuffer((d / "rgb_tiles.u8").read_bytes(), np.uint8),
                          O.warp_rgb(rgb, tiles))
    sm = np.frombuffer((d / "smooth.u16").read_bytes(), np.uint16).reshape(out_w // 2, out_w)
    assert np.array_equal(sm, O.solve_smoothing(tiles, warped, out_w, out_w // 2, zr))
