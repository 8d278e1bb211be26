"""ctypes wrapper of oracle/csrc/fold_ref.c (TEST INFRASTRUCTURE / CPU BASELINE ONLY)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libddsref.so")


def build():
    subprocess.run(["make", "-C", HERE], check=True, stdout=subprocess.DEVNULL)


def _lib():
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    lib.ddsref_fold.restype = C.c_int
    lib.ddsref_fold.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_size_t, C.c_char_p]
    return lib


def fold_be(mod_be: bytes, ops_be: bytes, width: int, count: int) -> bytes:
    lib = _lib()
    out = C.create_string_buffer(max(len(mod_be), width))
    rc = lib.ddsref_fold(mod_be, len(mod_be), ops_be, width, count, out)
    if rc:
        raise ValueError(f"ddsref_fold rc={rc}")
    return out.raw[: (width if count == 1 else len(mod_be))]


def fold(N: int, xs) -> int:
    mb = (N.bit_length() + 7) // 8
    width = max([mb] + [(int(x).bit_length() + 7) // 8 for x in xs])
    ops = b"".join(int(x).to_bytes(width, "big") for x in xs)
    return int.from_bytes(fold_be(N.to_bytes(mb, "big"), ops, width, len(xs)), "big")
