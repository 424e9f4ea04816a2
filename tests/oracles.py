"""Test-side access to the CPU checkers under oracle/ (test infrastructure only).

* ``orc``  -- oracle/liboracle.so, this repo's C restatement of the reference path;
* ``ref``  -- oracle/_ref/libbz2_ref.so, the reference library compiled from /root/reference
  by oracle/Makefile (travels prebuilt to the GPU box; None when it was never built).
The oracle delegates one value -- origPtr of exactly periodic blocks -- to
the reference build through orc_set_resolver.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORC_PATH = os.path.join(ORACLE_DIR, "liboracle.so")
REF_PATH = os.path.join(ORACLE_DIR, "_ref", "libbz2_ref.so")

_orc = None
_ref = None


def build_oracle():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def orc():
    global _orc
    if _orc is None:
        if not os.path.exists(ORC_PATH):
            build_oracle()
        L = ctypes.CDLL(ORC_PATH)
        vp, u64, ci = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
        L.orc_compress.restype = ctypes.c_int64
        L.orc_compress.argtypes = [vp, u64, ci, ci, vp, u64]
        L.orc_rle1.restype = ctypes.c_int64
        L.orc_rle1.argtypes = [vp, u64, ci, ci, vp, u64, vp, vp, ctypes.c_int64]
        L.orc_bwt.argtypes = [vp, ci, vp, ctypes.POINTER(ctypes.c_int)]
        L.orc_mtf.argtypes = [vp, ci, vp, vp, ctypes.POINTER(ctypes.c_int)]
        L.orc_code_lengths.argtypes = [vp, vp, ci, ci]
        L.orc_crc_table.restype = ctypes.c_uint32
        L.orc_crc_update.restype = ctypes.c_uint32
        L.orc_crc_update.argtypes = [ctypes.c_uint32, vp, u64]
        L.orc_set_resolver.argtypes = [vp]
        r = ref()
        if r is not None:
            L.orc_set_resolver(ctypes.cast(r.ref_blocksort, vp))
        _orc = L
    return _orc


def ref():
    global _ref
    if _ref is None and os.path.exists(REF_PATH):
        L = ctypes.CDLL(REF_PATH)
        vp, ci = ctypes.c_void_p, ctypes.c_int
        L.BZ2_bzBuffToBuffCompress.argtypes = [vp, ctypes.POINTER(ctypes.c_uint), vp, ctypes.c_uint, ci, ci, ci]
        L.ref_blocksort.argtypes = [vp, ci, vp]
        L.ref_hb_code_lengths.argtypes = [vp, vp, ci, ci]
        L.ref_crc_table_entry.restype = ctypes.c_uint32
        _ref = L
    return _ref


def has_ref():
    return ref() is not None


# ------------------------------------------------------------------ oracle wrappers
def orc_compress(data: bytes, level: int, tail_merge: int = 1) -> bytes:
    cap = len(data) * 2 + 4096
    out = ctypes.create_string_buffer(cap)
    n = orc().orc_compress(data, len(data), level, tail_merge, out, cap)
    assert n >= 0, "oracle failed (periodic block without resolver?)"
    return out.raw[:n]


def orc_rle1(data: bytes, level: int, tail_merge: int = 1):
    cap = len(data) + len(data) // 4 + 64
    blocks = ctypes.create_string_buffer(cap)
    maxb = len(data) // 90000 + 8
    off = (ctypes.c_uint64 * (maxb + 1))()
    crc = (ctypes.c_uint32 * maxb)()
    nb = orc().orc_rle1(data, len(data), level, tail_merge, blocks, cap, off, crc, maxb)
    assert nb >= 0
    offs = [off[i] for i in range(nb + 1)] if nb else [0]
    return blocks.raw[: offs[-1]], offs, [crc[i] for i in range(nb)]


def orc_bwt(block: bytes):
    n = len(block)
    out = ctypes.create_string_buffer(max(n, 1))
    per = ctypes.c_int(0)
    o = orc().orc_bwt(block, n, out, ctypes.byref(per))
    return out.raw[:n], o, per.value


def orc_mtf(bwt: bytes):
    n = len(bwt)
    mtfv = (ctypes.c_uint16 * (n + 2))()
    freq = (ctypes.c_int32 * 258)()
    nu = ctypes.c_int(0)
    nm = orc().orc_mtf(bwt, n, mtfv, freq, ctypes.byref(nu))
    return np.frombuffer(mtfv, dtype=np.uint16, count=nm).copy(), np.frombuffer(freq, dtype=np.int32).copy(), nu.value


def orc_code_lengths(freq, max_len=17):
    alpha = len(freq)
    f = (ctypes.c_int32 * alpha)(*freq)
    ln = (ctypes.c_int32 * alpha)()
    orc().orc_code_lengths(ln, f, alpha, max_len)
    return list(ln)


# ------------------------------------------------------------------ reference wrappers
def ref_compress(data: bytes, level: int) -> bytes:
    cap = len(data) + len(data) // 50 + 4096
    dst = ctypes.create_string_buffer(cap)
    dl = ctypes.c_uint(cap)
    rc = ref().BZ2_bzBuffToBuffCompress(dst, ctypes.byref(dl), data, len(data), level, 0, 30)
    assert rc == 0, rc
    return dst.raw[: dl.value]


def ref_decompress(data: bytes, cap: int, small: int = 0):
    """The reference's BZ2_bzBuffToBuffDecompress: (return code, output bytes)."""
    L = ref()
    dst = ctypes.create_string_buffer(max(cap, 1))
    dl = ctypes.c_uint(cap)
    L.BZ2_bzBuffToBuffDecompress.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint), ctypes.c_void_p,
                                             ctypes.c_uint, ctypes.c_int, ctypes.c_int]
    rc = L.BZ2_bzBuffToBuffDecompress(dst, ctypes.byref(dl), data, len(data), small, 0)
    return rc, dst.raw[: dl.value] if rc == 0 else b""


class _Strm(ctypes.Structure):
    _fields_ = [
        ("next_in", ctypes.c_void_p), ("avail_in", ctypes.c_uint),
        ("total_in_lo32", ctypes.c_uint), ("total_in_hi32", ctypes.c_uint),
        ("next_out", ctypes.c_void_p), ("avail_out", ctypes.c_uint),
        ("total_out_lo32", ctypes.c_uint), ("total_out_hi32", ctypes.c_uint),
        ("state", ctypes.c_void_p),
        ("bzalloc", ctypes.c_void_p), ("bzfree", ctypes.c_void_p), ("opaque", ctypes.c_void_p),
    ]


def ref_stream_compress(chunks, level: int, finish_with_last=False, flush_after=()) -> bytes:
    """The reference's own BZ2_bzCompress driven with the given call pattern."""
    L = ref()
    strm = _Strm()
    assert L.BZ2_bzCompressInit(ctypes.byref(strm), level, 0, 30) == 0
    ob = ctypes.create_string_buffer(1 << 16)
    out = bytearray()
    keep = []

    def pump(action):
        strm.next_out = ctypes.cast(ob, ctypes.c_void_p)
        strm.avail_out = 1 << 16
        r = L.BZ2_bzCompress(ctypes.byref(strm), action)
        out.extend(ob.raw[: (1 << 16) - strm.avail_out])
        assert r >= 0, r
        return r

    chunks = list(chunks)
    for i, c in enumerate(chunks):
        b = ctypes.create_string_buffer(bytes(c), len(c))
        keep[:] = [b]  # only the chunk being consumed (4 GiB inputs come in 256 MiB chunks)
        strm.next_in = ctypes.cast(b, ctypes.c_void_p)
        strm.avail_in = len(c)
        if finish_with_last and i == len(chunks) - 1:
            break
        while strm.avail_in > 0:
            pump(0)
        if i in flush_after:
            while pump(1) != 1:
                pass
    if not (finish_with_last and chunks):
        strm.avail_in = 0
    while pump(2) != 4:
        pass
    L.BZ2_bzCompressEnd(ctypes.byref(strm))
    return bytes(out)


def ref_blocksort(block: bytes):
    n = len(block)
    out = ctypes.create_string_buffer(max(n, 1))
    o = ref().ref_blocksort(block, n, out)
    return out.raw[:n], o


def ref_code_lengths(freq, max_len=17):
    alpha = len(freq)
    f = (ctypes.c_int32 * alpha)(*freq)
    ln = (ctypes.c_int32 * alpha)()
    ref().ref_hb_code_lengths(ln, f, alpha, max_len)
    return list(ln)
