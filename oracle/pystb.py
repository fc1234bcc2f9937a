"""ctypes binding of oracle/_ref/libstbref.so: the reference's own stb_image v2.23 /
stb_image_write v1.15, compiled from /root/reference by oracle/Makefile (see stb_ref.c).

TEST INFRASTRUCTURE ONLY -- the checker for the facade's image codecs (tests/test_codecs_stb.py,
tools/make_stb_golden.py); never imported by the product path.  available() is False where the
library was not built (no /root/reference at build time)."""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_ref", "libstbref.so")
_lib = None


def available():
    return os.path.exists(LIB_PATH)


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(LIB_PATH)
        ip = C.POINTER(C.c_int)
        L.sref_load.argtypes = [C.c_char_p, C.c_int, C.c_void_p, C.c_longlong, ip, ip, ip]
        L.sref_is_16_bit.argtypes = [C.c_char_p]
        L.sref_write_jpg.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int,
                                     C.POINTER(C.c_uint8), C.c_int, C.c_int]
        L.sref_failure_reason.restype = C.c_char_p
        _lib = L
    return _lib


def is_16_bit(fn):
    return bool(lib().sref_is_16_bit(str(fn).encode()))


def load(fn, want16=None):
    """stbi_load / stbi_load_16(fn, req_comp 0) -> [h][w][c] uint8 / uint16, or None on failure
    (want16 None: as the reference's Load decides, by stbi_is_16_bit)."""
    if want16 is None:
        want16 = is_16_bit(fn)
    w, h, c = C.c_int(), C.c_int(), C.c_int()
    cap = 1 << 26
    buf = np.zeros(cap, np.uint8)
    rc = lib().sref_load(str(fn).encode(), int(want16), buf.ctypes.data, cap, C.byref(w),
                         C.byref(h), C.byref(c))
    if rc == -2:
        n = w.value * h.value * c.value * (2 if want16 else 1)
        buf = np.zeros(n, np.uint8)
        rc = lib().sref_load(str(fn).encode(), int(want16), buf.ctypes.data, n, C.byref(w),
                             C.byref(h), C.byref(c))
    if rc:
        return None
    n = w.value * h.value * c.value
    a = buf[:n * (2 if want16 else 1)]
    a = a.view(np.uint16) if want16 else a
    return a.reshape(h.value, w.value, c.value).copy()


def write_jpg(fn, px, quality, flip=False):
    px = np.ascontiguousarray(px, np.uint8)
    h, w = px.shape[:2]
    c = 1 if px.ndim == 2 else px.shape[2]
    return lib().sref_write_jpg(str(fn).encode(), w, h, c, px.ctypes.data_as(C.POINTER(C.c_uint8)),
                                int(quality), int(flip))
