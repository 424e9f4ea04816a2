"""bzip2_amd -- MI355X-native bzip2 compression (drop-in libbz2) -- Python host mirror.

The product is the C-ABI shared library ``libbz2_amd.so`` built in this directory (SONAME
``libbz2.so.1.0``): it exports the reference's 24 ``bzlib.h`` functions (reference
libbz2.def:4-27) with the compression hot path on the GPU, plus the ``bzg_*`` engine entry
points of ``include/bzg.h``.  This module binds both with ctypes so that tests and the
benchmark call exactly what a C caller would call.

There is no CPU fallback: if the library or a usable GPU is missing, compression raises.
"""
from __future__ import annotations

import ctypes
import os

try:  # share torch's HIP runtime (its libamdhip64 carries SONAME libamdhip64.so.7)
    import torch as _torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the C ABI
    _torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
# BZ2_AMD_LIB: an alternative in-tree build of the same library (development A/B runs)
LIB_PATH = os.environ.get("BZ2_AMD_LIB") or os.path.join(HERE, "libbz2_amd.so")

# bzlib.h return codes (reference bzlib.h:33-46)
BZ_RUN, BZ_FLUSH, BZ_FINISH = 0, 1, 2
BZ_OK, BZ_RUN_OK, BZ_FLUSH_OK, BZ_FINISH_OK, BZ_STREAM_END = 0, 1, 2, 3, 4
BZ_SEQUENCE_ERROR, BZ_PARAM_ERROR, BZ_MEM_ERROR = -1, -2, -3
BZ_DATA_ERROR, BZ_DATA_ERROR_MAGIC, BZ_IO_ERROR = -4, -5, -6
BZ_UNEXPECTED_EOF, BZ_OUTBUFF_FULL, BZ_CONFIG_ERROR = -7, -8, -9

BZG_FLAG_END_SEGMENT, BZG_FLAG_TAIL_MERGE, BZG_FLAG_TRAILER = 1, 2, 4

EXPORTS = [
    "BZ2_bzCompressInit", "BZ2_bzCompress", "BZ2_bzCompressEnd",
    "BZ2_bzDecompressInit", "BZ2_bzDecompress", "BZ2_bzDecompressEnd",
    "BZ2_bzReadOpen", "BZ2_bzReadClose", "BZ2_bzReadGetUnused", "BZ2_bzRead",
    "BZ2_bzWriteOpen", "BZ2_bzWrite", "BZ2_bzWriteClose", "BZ2_bzWriteClose64",
    "BZ2_bzBuffToBuffCompress", "BZ2_bzBuffToBuffDecompress", "BZ2_bzlibVersion",
    "BZ2_bzopen", "BZ2_bzdopen", "BZ2_bzread", "BZ2_bzwrite", "BZ2_bzflush",
    "BZ2_bzclose", "BZ2_bzerror",
]
ENGINE_EXPORTS = [
    "bzg_stream_init", "bzg_compress_device", "bzg_compress_host", "bzg_compress_host_stream",
    "bzg_bound", "bzg_stage_rle1", "bzg_stage_bwt", "bzg_stage_mtf", "bzg_stage_code_lengths", "bzg_last_stats",
    "bzg_release", "bzg_device_ok", "bzg_periodic_origptr", "bzg_copy_rank_closed_form", "bzg_qperiodic_bwt", "bzg_seg_map", "bzg_seg_walk",
    "bzg_find_magics", "bzg_decompress_device", "bzg_decompress_host", "bzg_last_decode_stats",
]


class BzError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        super().__init__(f"{what}: bzlib error {code}")
        self.code = code


class bz_stream(ctypes.Structure):
    """Byte-identical to the reference's bz_stream (bzlib.h:48-66)."""

    _fields_ = [
        ("next_in", ctypes.c_void_p), ("avail_in", ctypes.c_uint),
        ("total_in_lo32", ctypes.c_uint), ("total_in_hi32", ctypes.c_uint),
        ("next_out", ctypes.c_void_p), ("avail_out", ctypes.c_uint),
        ("total_out_lo32", ctypes.c_uint), ("total_out_hi32", ctypes.c_uint),
        ("state", ctypes.c_void_p),
        ("bzalloc", ctypes.c_void_p), ("bzfree", ctypes.c_void_p), ("opaque", ctypes.c_void_p),
    ]


class bzg_stream_state(ctypes.Structure):
    _fields_ = [
        ("combined_crc", ctypes.c_uint32), ("blocks_done", ctypes.c_uint32),
        ("carry_byte", ctypes.c_uint8), ("carry_bits", ctypes.c_uint8),
        ("header_done", ctypes.c_uint8), ("level", ctypes.c_uint8),
    ]


class bzg_stats(ctypes.Structure):
    _fields_ = [
        ("rle1_ms", ctypes.c_float), ("bwt_ms", ctypes.c_float), ("mtf_ms", ctypes.c_float),
        ("code_ms", ctypes.c_float), ("total_ms", ctypes.c_float),
        ("nblocks", ctypes.c_uint32), ("sort_iterations", ctypes.c_uint32),
        ("rle_bytes", ctypes.c_uint64), ("sort_unsorted", ctypes.c_uint64),
        ("mtf_symbols", ctypes.c_uint64), ("a5_roots", ctypes.c_uint32), ("a5_host", ctypes.c_uint32),
    ]


class bzg_decode_stats(ctypes.Structure):
    _fields_ = [
        ("total_ms", ctypes.c_float), ("blocks", ctypes.c_uint64), ("candidates", ctypes.c_uint64),
        ("out_bytes", ctypes.c_uint64),
    ]


_lib = None


def lib() -> ctypes.CDLL:
    """The product library; raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C {HERE}` or __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        u64, u32, vp, ci = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int
        L.BZ2_bzBuffToBuffCompress.argtypes = [vp, ctypes.POINTER(ctypes.c_uint), vp, ctypes.c_uint, ci, ci, ci]
        L.BZ2_bzBuffToBuffDecompress.argtypes = [vp, ctypes.POINTER(ctypes.c_uint), vp, ctypes.c_uint, ci, ci]
        L.BZ2_bzCompressInit.argtypes = [ctypes.POINTER(bz_stream), ci, ci, ci]
        L.BZ2_bzCompress.argtypes = [ctypes.POINTER(bz_stream), ci]
        L.BZ2_bzCompressEnd.argtypes = [ctypes.POINTER(bz_stream)]
        L.BZ2_bzDecompressInit.argtypes = [ctypes.POINTER(bz_stream), ci, ci]
        L.BZ2_bzDecompress.argtypes = [ctypes.POINTER(bz_stream)]
        L.BZ2_bzDecompressEnd.argtypes = [ctypes.POINTER(bz_stream)]
        L.BZ2_bzlibVersion.restype = ctypes.c_char_p
        L.bzg_stream_init.argtypes = [ctypes.POINTER(bzg_stream_state), ci]
        L.bzg_compress_device.argtypes = [vp, u64, ctypes.c_uint, ctypes.POINTER(bzg_stream_state), vp, u64,
                                          ctypes.POINTER(u64), ctypes.POINTER(u64), vp]
        L.bzg_compress_host.argtypes = [vp, u64, ci, vp, u64, ctypes.POINTER(u64)]
        L.bzg_bound.argtypes = [u64]
        L.bzg_bound.restype = u64
        L.bzg_stage_rle1.argtypes = [vp, u64, ci, ci, vp, u64, vp, vp, ctypes.POINTER(u32), u32]
        L.bzg_stage_bwt.argtypes = [vp, vp, u32, vp, vp]
        L.bzg_stage_mtf.argtypes = [vp, vp, u32, vp, ctypes.c_uint64, vp, vp, vp]
        L.bzg_stage_code_lengths.argtypes = [vp, vp, u32, ci, vp]
        L.bzg_last_stats.argtypes = [ctypes.POINTER(bzg_stats)]
        L.bzg_periodic_origptr.argtypes = [vp, ctypes.c_int32]
        L.bzg_seg_map.argtypes = [vp, u64, ci, vp]
        L.bzg_find_magics.argtypes = [vp, u64, vp, u64, ctypes.POINTER(u64), vp]
        L.bzg_seg_walk.argtypes = [u32, ci, vp, u32, ctypes.POINTER(u32), ctypes.POINTER(u64), ctypes.POINTER(u32)]
        L.bzg_periodic_origptr.restype = ctypes.c_int32
        L.bzg_copy_rank_closed_form.argtypes = [vp, ctypes.c_int32, ctypes.c_int32]
        L.bzg_copy_rank_closed_form.restype = ctypes.c_int32
        L.bzg_qperiodic_bwt.argtypes = [vp, u32, vp, ctypes.POINTER(u32)]
        L.bzg_qperiodic_bwt.restype = u32
        L.bzg_decompress_device.argtypes = [vp, u64, vp, u64, ctypes.POINTER(u64), vp]
        L.bzg_decompress_host.argtypes = [vp, u64, vp, u64, ctypes.POINTER(u64)]
        L.bzg_last_decode_stats.argtypes = [ctypes.POINTER(bzg_decode_stats)]
        _lib = L
    return _lib


def device_ok() -> bool:
    return bool(lib().bzg_device_ok())


def version() -> str:
    return lib().BZ2_bzlibVersion().decode()


def bound(n: int) -> int:
    return int(lib().bzg_bound(n))


def buff_to_buff_compress(data: bytes, level: int = 9) -> bytes:
    """BZ2_bzBuffToBuffCompress (reference bzlib.c:1309-1357): FINISH with all input."""
    src = bytes(data)
    cap = bound(len(src))
    dst = ctypes.create_string_buffer(cap)
    dl = ctypes.c_uint(cap)
    rc = lib().BZ2_bzBuffToBuffCompress(dst, ctypes.byref(dl), src, len(src), level, 0, 30)
    if rc != BZ_OK:
        raise BzError(rc, "BZ2_bzBuffToBuffCompress")
    return dst.raw[: dl.value]


def buff_to_buff_decompress(data: bytes, out_cap: int, small: int = 0) -> bytes:
    """BZ2_bzBuffToBuffDecompress (reference bzlib.c:1361-1410): the GPU decoder for small=0
    when a device is present, the library's bit-serial decoder otherwise."""
    dst = ctypes.create_string_buffer(max(out_cap, 1))
    dl = ctypes.c_uint(out_cap)
    rc = lib().BZ2_bzBuffToBuffDecompress(dst, ctypes.byref(dl), bytes(data), len(data), small, 0)
    if rc != BZ_OK:
        raise BzError(rc, "BZ2_bzBuffToBuffDecompress")
    return dst.raw[: dl.value]


def decompress_device(d_in_ptr: int, n: int, d_out_ptr: int, out_cap: int, stream_ptr: int = 0):
    """bzg_decompress_device on device-resident buffers: (return code, bytes written)."""
    got = ctypes.c_uint64(0)
    rc = lib().bzg_decompress_device(ctypes.c_void_p(d_in_ptr), n, ctypes.c_void_p(d_out_ptr), out_cap,
                                     ctypes.byref(got), ctypes.c_void_p(stream_ptr or None))
    return rc, got.value


def decompress_host(data: bytes, out_cap: int):
    """bzg_decompress_host: (return code, output bytes)."""
    dst = ctypes.create_string_buffer(max(out_cap, 1))
    got = ctypes.c_uint64(0)
    rc = lib().bzg_decompress_host(bytes(data), len(data), dst, out_cap, ctypes.byref(got))
    return rc, dst.raw[: got.value]


def last_decode_stats() -> dict:
    s = bzg_decode_stats()
    lib().bzg_last_decode_stats(ctypes.byref(s))
    return {k: getattr(s, k) for k, _ in bzg_decode_stats._fields_}


def stream_compress(chunks, level: int = 9, finish_with_last: bool = False, out_chunk: int = 1 << 16,
                    flush_after=(), progress=None) -> bytes:
    """Drive BZ2_bzCompress like a streaming caller: every chunk with BZ_RUN (or, for the last
    chunk when finish_with_last, with BZ_FINISH directly), then BZ_FINISH until
    BZ_STREAM_END.  Chunk indices listed in flush_after are followed by BZ_FLUSH.  A list
    passed as progress receives (input bytes given, output bytes received) after each RUN
    chunk."""
    L = lib()
    strm = bz_stream()
    rc = L.BZ2_bzCompressInit(ctypes.byref(strm), level, 0, 30)
    if rc != BZ_OK:
        raise BzError(rc, "BZ2_bzCompressInit")
    out = bytearray()
    obuf = ctypes.create_string_buffer(out_chunk)
    keep = []

    def pump(action, expect):
        while True:
            strm.next_out = ctypes.cast(obuf, ctypes.c_void_p)
            strm.avail_out = out_chunk
            r = L.BZ2_bzCompress(ctypes.byref(strm), action)
            out.extend(obuf.raw[: out_chunk - strm.avail_out])
            if r not in expect:
                raise BzError(r, f"BZ2_bzCompress({action})")
            return r

    try:
        chunks = list(chunks)
        for i, c in enumerate(chunks):
            buf = ctypes.create_string_buffer(bytes(c), len(c))
            keep.append(buf)
            strm.next_in = ctypes.cast(buf, ctypes.c_void_p)
            strm.avail_in = len(c)
            if finish_with_last and i == len(chunks) - 1:
                break
            while strm.avail_in > 0:
                pump(BZ_RUN, (BZ_RUN_OK,))
            if progress is not None:
                progress.append((sum(len(x) for x in chunks[: i + 1]), len(out)))
            if i in flush_after:
                while pump(BZ_FLUSH, (BZ_FLUSH_OK, BZ_RUN_OK)) != BZ_RUN_OK:
                    pass
        if not (finish_with_last and chunks):
            strm.avail_in = 0
        while pump(BZ_FINISH, (BZ_FINISH_OK, BZ_STREAM_END)) != BZ_STREAM_END:
            pass
    finally:
        L.BZ2_bzCompressEnd(ctypes.byref(strm))
    return bytes(out)


def compress_device(d_in_ptr: int, n: int, level: int, d_out_ptr: int, out_cap: int, *, flags=None,
                    state: bzg_stream_state | None = None, stream_ptr: int = 0):
    """bzg_compress_device on device-resident buffers.  Returns (out_bytes, consumed, state)."""
    L = lib()
    st = state if state is not None else bzg_stream_state()
    if state is None:
        L.bzg_stream_init(ctypes.byref(st), level)
    if flags is None:
        flags = BZG_FLAG_END_SEGMENT | BZG_FLAG_TRAILER | (BZG_FLAG_TAIL_MERGE if n else 0)
    ob = ctypes.c_uint64(0)
    cons = ctypes.c_uint64(0)
    rc = L.bzg_compress_device(ctypes.c_void_p(d_in_ptr), n, flags, ctypes.byref(st), ctypes.c_void_p(d_out_ptr),
                               out_cap, ctypes.byref(ob), ctypes.byref(cons), ctypes.c_void_p(stream_ptr or None))
    if rc != BZ_OK:
        raise BzError(rc, "bzg_compress_device")
    return ob.value, cons.value, st


def seg_map(d_ptr: int, n: int, level: int, stream_ptr: int = 0) -> None:
    """bzg_seg_map: RLE1 chunk map of a device region that starts at a chunk start."""
    rc = lib().bzg_seg_map(ctypes.c_void_p(d_ptr), n, level, ctypes.c_void_p(stream_ptr or None))
    if rc != BZ_OK:
        raise BzError(rc, "bzg_seg_map")


def seg_walk(fill_in: int, final_region: bool, max_cuts: int):
    """bzg_seg_walk over the last mapped region: (cuts, last_chunk, last_fill), region-relative."""
    cuts = (ctypes.c_uint64 * max(1, max_cuts))()
    nc, lc, lf = ctypes.c_uint32(0), ctypes.c_uint64(0), ctypes.c_uint32(0)
    rc = lib().bzg_seg_walk(fill_in, 1 if final_region else 0, cuts, max_cuts, ctypes.byref(nc), ctypes.byref(lc),
                            ctypes.byref(lf))
    if rc != BZ_OK:
        raise BzError(rc, "bzg_seg_walk")
    return [int(cuts[i]) for i in range(nc.value)], lc.value, lf.value


def find_magics(d_ptr: int, n: int, stream_ptr: int = 0):
    """bzg_find_magics on a device buffer: sorted [(bit_offset, kind)], kind 0 = block header,
    1 = end of stream."""
    L = lib()
    cnt = ctypes.c_uint64(0)
    cap = n // 4096 + 1024
    while True:
        out = (ctypes.c_uint64 * cap)()
        rc = L.bzg_find_magics(ctypes.c_void_p(d_ptr), n, out, cap, ctypes.byref(cnt), ctypes.c_void_p(stream_ptr or None))
        if rc == BZ_OUTBUFF_FULL:
            cap = cnt.value
            continue
        if rc != BZ_OK:
            raise BzError(rc, "bzg_find_magics")
        return [(out[i] >> 1, out[i] & 1) for i in range(cnt.value)]


def code_lengths(tables, max_len: int = 17):
    """BZ2_hbMakeCodeLengths (reference huffman.c:63-148) on the GPU for a list of frequency
    tables (2..258 counts each); returns the code lengths per table."""
    n = len(tables)
    freq = (ctypes.c_uint32 * (max(n, 1) * 258))()
    alpha = (ctypes.c_int32 * max(n, 1))()
    for t, f in enumerate(tables):
        alpha[t] = len(f)
        for i, v in enumerate(f):
            freq[t * 258 + i] = v
    lens = (ctypes.c_uint8 * (max(n, 1) * 258))()
    rc = lib().bzg_stage_code_lengths(freq, alpha, n, max_len, lens)
    if rc != BZ_OK:
        raise BzError(rc, "bzg_stage_code_lengths")
    return [[lens[t * 258 + i] for i in range(len(f))] for t, f in enumerate(tables)]


def periodic_origptr(block: bytes) -> int:
    """origPtr the reference assigns to an exactly periodic block (host replay, A5)."""
    return int(lib().bzg_periodic_origptr(bytes(block), len(block)))


def copy_rank_closed_form(root: bytes, k: int) -> int:
    """The copy rank the device computes in closed form for root^k (origptr.hip's rules), or -1
    when the host model decides (A5; host mirror, no GPU)."""
    return int(lib().bzg_copy_rank_closed_form(bytes(root), len(root), k))


def qperiodic_bwt(block: bytes):
    """(period, BWT, origPtr) of a quasi-periodic block by the analytic order the GPU sort
    uses for it (qsa.cpp, host); None when the block is not quasi-periodic."""
    n = len(block)
    out = ctypes.create_string_buffer(max(n, 1))
    o = ctypes.c_uint32(0)
    p = int(lib().bzg_qperiodic_bwt(bytes(block), n, out, ctypes.byref(o)))
    return (p, out.raw[:n], o.value) if p else None


def last_stats() -> dict:
    s = bzg_stats()
    lib().bzg_last_stats(ctypes.byref(s))
    return {k: getattr(s, k) for k, _ in bzg_stats._fields_}
