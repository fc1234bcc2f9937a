"""CPU checks of the C-ABI boundary: libpanofuse.so loads, exports every function that
include/panofuse.h declares, and its pure-host entry points agree with the oracle.  No device
calls are made here (there is no GPU in the build container)."""
import ctypes as C
import os
import re

import pytest

import panofuse
import pf_layouts as PL
import pyoracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "panofuse.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pf_[a-z0-9_]+)\s*\(", src)))


def test_header_matches_binding_list():
    assert _declared() == sorted(panofuse.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(panofuse.LIB_PATH)
    for name in _declared():
        assert hasattr(lib, name), name
    assert panofuse.load().pf_version().startswith(b"panofuse")


def test_library_is_gfx950_code_object():
    data = open(panofuse.LIB_PATH, "rb").read()
    assert b"gfx950" in data


@pytest.mark.parametrize("out_w", [512, 2048, 4096, 8192])
def test_level_info_matches_oracle(out_w):
    zr = PL.ZENITH_RANGE
    for level in range(O.num_levels(out_w)):
        lv = O.level_dims(out_w, out_w // 2, zr, level)
        got = panofuse.level_info(out_w, out_w // 2, zr, level)
        assert got == (lv.w, lv.h, lv.h0, lv.h1, lv.iters, lv.max_level)


def test_level_info_rejects_bad_level():
    with pytest.raises(panofuse.PanofuseError):
        panofuse.level_info(2048, 1024, PL.ZENITH_RANGE, 3)


def test_fuser_refuses_without_gpu():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        panofuse.Fuser(0)
