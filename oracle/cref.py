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


# ---- OpenSSL BIGNUM baselines (oracle/csrc/bn_baseline.c) ----
BNLIB = os.path.join(HERE, "build", "libbnref.so")


def _bnlib():
    if not os.path.exists(BNLIB):
        build()
    lib = C.CDLL(BNLIB)
    lib.bnref_fold.restype = C.c_int
    lib.bnref_fold.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_size_t, C.c_int, C.c_char_p]
    lib.bnref_paillier_encrypt.restype = C.c_int
    lib.bnref_paillier_encrypt.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_void_p, C.c_char_p,
                                           C.c_size_t, C.c_size_t, C.c_int, C.c_char_p, C.c_size_t]
    return lib


def bn_fold_be(mod_be: bytes, ops_be: bytes, width: int, count: int, threads: int = 1) -> bytes:
    out = C.create_string_buffer(len(mod_be))
    rc = _bnlib().bnref_fold(mod_be, len(mod_be), ops_be, width, count, threads, out)
    if rc:
        raise ValueError(f"bnref_fold rc={rc}")
    return out.raw


def bn_paillier_encrypt(n: int, g: int, ms, rs, threads: int = 1) -> list:
    import numpy as np
    nb, gb = (n.bit_length() + 7) // 8, (g.bit_length() + 7) // 8
    nsqb = ((n * n).bit_length() + 7) // 8
    rw = max([1] + [(int(r).bit_length() + 7) // 8 for r in rs])
    m = np.ascontiguousarray(ms, dtype=np.uint32)
    out = C.create_string_buffer(nsqb * max(1, len(rs)))
    rc = _bnlib().bnref_paillier_encrypt(n.to_bytes(nb, "big"), nb, g.to_bytes(gb, "big"), gb,
                                         m.ctypes.data_as(C.c_void_p), b"".join(int(r).to_bytes(rw, "big") for r in rs),
                                         rw, len(rs), threads, out, nsqb)
    if rc:
        raise ValueError(f"bnref_paillier_encrypt rc={rc}")
    raw = out.raw
    return [int.from_bytes(raw[i * nsqb:(i + 1) * nsqb], "big") for i in range(len(rs))]
