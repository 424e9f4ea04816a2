"""CPU tests of the drop-in boundary: the product library builds for gfx950, loads without a
GPU, and exports every symbol include/*.h declares (libbz2.def:4-27 plus the bzg_* engine ABI).
No compute calls here (no GPU in this container)."""
import ctypes
import os
import re
import subprocess

import pytest

import bzip2_amd
import bzip2_amd as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions(path):
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = set(re.findall(r"BZ_API\((BZ2_\w+)\)", txt))
    names |= set(re.findall(r"^\s*[\w\s\*]+?\b(bzg_\w+)\s*\(", txt, flags=re.M))
    return names


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(bzip2_amd.LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "bzip2_amd")], check=True)
    return bzip2_amd.lib()


def test_exports_match_reference_def(lib):
    ref_def = [l.strip() for l in open(os.path.join(ROOT, "tests", "golden", "libbz2.def.txt"))]
    assert sorted(ref_def) == sorted(bzip2_amd.EXPORTS)
    for name in bzip2_amd.EXPORTS + bzip2_amd.ENGINE_EXPORTS:
        assert hasattr(lib, name), name


def test_every_header_symbol_is_exported(lib):
    declared = header_functions(os.path.join(ROOT, "include", "bzlib.h"))
    declared |= header_functions(os.path.join(ROOT, "include", "bzg.h"))
    assert len(declared) >= 24 + 10
    out = subprocess.run(["nm", "-D", "--defined-only", bzip2_amd.LIB_PATH], capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = declared - exported
    assert not missing, missing


def test_soname_is_drop_in(lib):
    out = subprocess.run(["readelf", "-d", bzip2_amd.LIB_PATH], capture_output=True, text=True).stdout
    assert "libbz2.so.1.0" in out


def test_version_string(lib):
    assert bzip2_amd.version() == "1.0.6x, 16-Aug-2018"


def test_bz_stream_layout():
    # bzlib.h:48-66 on LP64
    assert ctypes.sizeof(bzip2_amd.bz_stream) == 80
    assert bzip2_amd.bz_stream.state.offset == 48


def test_param_errors_without_gpu(lib):
    dl = ctypes.c_uint(100)
    buf = ctypes.create_string_buffer(100)
    assert lib.BZ2_bzBuffToBuffCompress(buf, ctypes.byref(dl), b"x", 1, 0, 0, 30) == bzip2_amd.BZ_PARAM_ERROR
    assert lib.BZ2_bzBuffToBuffCompress(buf, ctypes.byref(dl), b"x", 1, 10, 0, 30) == bzip2_amd.BZ_PARAM_ERROR
    assert lib.BZ2_bzBuffToBuffCompress(buf, ctypes.byref(dl), b"x", 1, 9, 5, 30) == bzip2_amd.BZ_PARAM_ERROR
    assert lib.BZ2_bzBuffToBuffCompress(buf, ctypes.byref(dl), b"x", 1, 9, 0, 251) == bzip2_amd.BZ_PARAM_ERROR
    assert lib.BZ2_bzCompressInit(None, 9, 0, 0) == bzip2_amd.BZ_PARAM_ERROR


def test_decoder_round_trips_reference_golden(lib):
    """The decompression half is this library's own CPU decoder; it must read the reference's
    golden streams."""
    for i in (1, 2, 3):
        comp = open(os.path.join(ROOT, "tests", "golden", f"sample{i}.bz2"), "rb").read()
        plain = open(os.path.join(ROOT, "tests", "golden", f"sample{i}.ref"), "rb").read()
        assert bzip2_amd.buff_to_buff_decompress(comp, len(plain) + 10) == plain


def test_decoder_streaming_small_chunks(lib):
    comp = open(os.path.join(ROOT, "tests", "golden", "sample1.bz2"), "rb").read()
    plain = open(os.path.join(ROOT, "tests", "golden", "sample1.ref"), "rb").read()
    L = lib
    strm = bzip2_amd.bz_stream()
    assert L.BZ2_bzDecompressInit(ctypes.byref(strm), 0, 0) == 0
    out = bytearray()
    ob = ctypes.create_string_buffer(777)
    tail = comp + b"TRAILING"
    inb = ctypes.create_string_buffer(tail, len(tail))
    pos = 0
    rc = 0
    while rc != bzip2_amd.BZ_STREAM_END:
        step = min(333, len(tail) - pos)
        strm.next_in = ctypes.c_void_p(ctypes.addressof(inb) + pos)
        strm.avail_in = step
        while True:
            strm.next_out = ctypes.cast(ob, ctypes.c_void_p)
            strm.avail_out = 777
            rc = L.BZ2_bzDecompress(ctypes.byref(strm))
            out += ob.raw[: 777 - strm.avail_out]
            assert rc in (0, 4), rc
            if rc == 4 or (strm.avail_out > 0 and strm.avail_in == 0):
                break
        pos += step - strm.avail_in
    L.BZ2_bzDecompressEnd(ctypes.byref(strm))
    assert bytes(out) == plain
    assert tail[pos:] == b"TRAILING"  # input consumed exactly to the end of the stream


def test_periodic_resolver_matches_reference(lib):
    """A5: origPtr of exactly periodic blocks (bzip2_amd/csrc/copyrank.cpp, with the closed
    form the device uses for one B* per period) against the reference build: the SURVEY.md 8a
    KATs and random periodic blocks."""
    from tests import oracles as O
    if not O.has_ref():
        pytest.skip("oracle/_ref not built")
    import random
    rng = random.Random(5)
    cases = [b"abc" * k for k in (2, 8, 16, 17, 100, 255, 256, 257, 1000, 4096)]
    cases += [b"abcabcabd" * k for k in (2, 8, 255, 1000)]
    cases += [b"bababac" * k for k in (16, 100, 256)]
    cases += [bytes([c] * 4 + [0xFB]) * 19997 for c in (0x00, 0x61, 0xFB, 0xFF)]
    for _ in range(200):
        w = bytes(rng.randrange(rng.choice([2, 4, 256])) for _ in range(rng.randint(1, 40)))
        cases.append(w * rng.randint(2, 300))
    for blk in cases:
        assert B.periodic_origptr(blk) == O.ref_blocksort(blk)[1], (blk[:12], len(blk))


def test_periodic_origptr_fuzz(lib):
    """5,000 random periodic blocks across the regimes of the tie model: short and long roots,
    2..60,000 copies, one-B*-per-period single-byte-run roots up to full 900 kB blocks (merge
    buffer in the text, in a 256-entry scratch, or the unsorted bucket rest)."""
    from tests import oracles as O
    if not O.has_ref():
        pytest.skip("oracle/_ref not built")
    import random
    rng = random.Random(20260)
    for _ in range(5000):
        mode = rng.random()
        if mode < 0.4:
            w = bytes(rng.randrange(rng.choice([2, 3, 4, 256])) for _ in range(rng.randint(1, 12)))
            k = rng.randint(2, 3000)
        elif mode < 0.7:
            w = bytes(rng.randrange(rng.choice([2, 4, 26, 256])) for _ in range(rng.randint(1, 60)))
            k = rng.randint(2, 200)
        elif mode < 0.9:
            w = bytes(rng.randrange(rng.choice([2, 4])) for _ in range(rng.randint(2, 6)))
            k = rng.randint(1000, 60000)
        else:
            w = bytes([rng.randrange(256)] * 4 + [rng.randrange(256)])
            k = rng.randint(2, 180000)
        blk = w * min(k, 900000 // len(w))
        assert B.periodic_origptr(blk) == O.ref_blocksort(blk)[1], (w, len(blk) // len(w))


def test_periodic_origptr_fuzz_wide(lib):
    """A5 copy-rank model on roots the short fuzz rarely draws: text-like roots up to 3,000
    bytes, dense binary/ternary roots with hundreds of B* offsets (the rank stage runs out of
    budget and finishes by doubling), near-periodic roots (classes with equal B* substrings),
    up to full 900 kB blocks."""
    from tests import datagen, oracles as O
    if not O.has_ref():
        pytest.skip("oracle/_ref not built")
    import random
    rng = random.Random(31337)
    txt = datagen.text(100_000, 77)
    for _ in range(160):
        mode = rng.random()
        if mode < 0.35:
            s = rng.randrange(0, len(txt) - 3000)
            w = txt[s:s + rng.randint(2, 3000)]
        elif mode < 0.7:
            w = bytes(rng.randrange(rng.choice([2, 3])) for _ in range(rng.randint(8, 400)))
        else:
            u = bytes(rng.randrange(4) for _ in range(rng.randint(1, 8)))
            w = u * rng.randint(2, 30) + bytes([rng.randrange(4)])
        k = rng.randint(2, max(2, 900_000 // len(w)))
        blk = (w * k)[:900_000]
        if len(set(blk)) == 1 or len(blk) < 2 * len(w):
            continue
        assert B.periodic_origptr(blk) == O.ref_blocksort(blk)[1], (len(w), w[:24], len(blk) // len(w))


def test_qperiodic_bwt_host_matches_oracle(lib):
    """Analytic order of quasi-periodic blocks (qsa.cpp, the plan the GPU sort writes out with
    k_qsa) against the oracle's BWT, and against the reference build when present: RLE1 shapes
    of a repeated byte, random roots of 2..256 bytes with every tail length class."""
    from tests import oracles as O
    import random
    rng = random.Random(2718)
    cases = [bytes([c] * 4 + [0xFB]) * k + bytes([c]) * r for c in (0, 0x61, 0xFF) for k in (2, 9, 4000)
             for r in (1, 2, 3)]
    for _ in range(200):
        w = bytes(rng.randrange(rng.choice([2, 3, 4, 256])) for _ in range(rng.randint(2, 256)))
        k = rng.randint(2, max(2, 12_000 // len(w)))
        cases.append(w * k + w[: rng.randint(1, len(w) - 1)])
    seen = 0
    for blk in cases:
        q = B.qperiodic_bwt(blk)
        if q is None:
            continue
        seen += 1
        L, o, per = O.orc_bwt(blk)
        assert per == len(blk)
        assert q[1:] == (L, o), (q[0], len(blk), blk[:12])
        if O.has_ref():
            assert q[1:] == O.ref_blocksort(blk), (q[0], len(blk))
    assert seen >= 200
    # not quasi-periodic: text, exact powers, periods above 256 or without two copies
    assert B.qperiodic_bwt(b"abcab" * 3) is None  # exact power
    assert B.qperiodic_bwt(bytes(range(200)) * 3 + b"\x00") is not None
    assert B.qperiodic_bwt(bytes(range(256)) + bytes([7]) + bytes(range(256)) + bytes([7]) + b"\x00") is None
    assert B.qperiodic_bwt(b"abcdefgh" + b"abc") is None


def _libc():
    c = ctypes.CDLL(None)
    c.fopen.restype = ctypes.c_void_p
    c.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    c.fclose.argtypes = [ctypes.c_void_p]
    return c


def _file_api(lib):
    vp, ip = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)
    lib.BZ2_bzReadOpen.restype = vp
    lib.BZ2_bzReadOpen.argtypes = [ip, vp, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int]
    lib.BZ2_bzRead.argtypes = [ip, vp, vp, ctypes.c_int]
    lib.BZ2_bzReadClose.argtypes = [ip, vp]
    lib.BZ2_bzReadGetUnused.argtypes = [ip, vp, ctypes.POINTER(vp), ip]
    lib.BZ2_bzopen.restype = vp
    lib.BZ2_bzopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    lib.BZ2_bzread.argtypes = [vp, vp, ctypes.c_int]
    lib.BZ2_bzclose.argtypes = [vp]
    lib.BZ2_bzerror.restype = ctypes.c_char_p
    lib.BZ2_bzerror.argtypes = [vp, ip]
    lib.BZ2_bzWriteOpen.restype = vp
    lib.BZ2_bzWriteOpen.argtypes = [ip, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    return lib


@pytest.mark.parametrize("i", [1, 2, 3])
def test_file_api_reads_reference_golden(lib, i, tmp_path):
    """BZ2_bzopen / BZ2_bzread / BZ2_bzerror / BZ2_bzclose (bzlib.c:1445-1628) and
    BZ2_bzReadOpen / bzRead / ReadGetUnused (bzlib.c:1149-1300) on the shipped goldens, with
    trailing bytes after the stream handed back as 'unused'."""
    L = _file_api(lib)
    g = os.path.join(ROOT, "tests", "golden")
    want = open(os.path.join(g, f"sample{i}.ref"), "rb").read()
    b = L.BZ2_bzopen(os.path.join(g, f"sample{i}.bz2").encode(), b"rb")
    assert b
    out = bytearray()
    buf = ctypes.create_string_buffer(7777)
    while True:
        n = L.BZ2_bzread(b, buf, 7777)
        assert n >= 0
        if n == 0:
            break
        out += buf.raw[:n]
    err = ctypes.c_int(1)
    assert L.BZ2_bzerror(b, ctypes.byref(err)) == b"OK" and err.value == 0  # STREAM_END (>0) reads as OK
    L.BZ2_bzclose(b)
    assert bytes(out) == want
    # trailing garbage comes back through BZ2_bzReadGetUnused
    p = tmp_path / "s.bz2"
    p.write_bytes(open(os.path.join(g, f"sample{i}.bz2"), "rb").read() + b"TRAILER")
    c = _libc()
    f = c.fopen(str(p).encode(), b"rb")
    e = ctypes.c_int(0)
    h = L.BZ2_bzReadOpen(ctypes.byref(e), f, 0, 0, None, 0)
    assert h and e.value == B.BZ_OK
    got = bytearray()
    big = ctypes.create_string_buffer(1 << 20)
    while e.value == B.BZ_OK:
        n = L.BZ2_bzRead(ctypes.byref(e), h, big, 1 << 20)
        got += big.raw[:n]
    assert e.value == B.BZ_STREAM_END and bytes(got) == want
    un, nun = ctypes.c_void_p(), ctypes.c_int(0)
    L.BZ2_bzReadGetUnused(ctypes.byref(e), h, ctypes.byref(un), ctypes.byref(nun))
    assert e.value == B.BZ_OK and ctypes.string_at(un, nun.value) == b"TRAILER"
    L.BZ2_bzReadClose(ctypes.byref(e), h)
    assert e.value == B.BZ_OK
    c.fclose(f)


def test_file_api_argument_errors(lib, tmp_path):
    L = _file_api(lib)
    e = ctypes.c_int(0)
    assert not L.BZ2_bzReadOpen(ctypes.byref(e), None, 0, 0, None, 0) and e.value == B.BZ_PARAM_ERROR
    c = _libc()
    p = tmp_path / "x"
    p.write_bytes(b"")
    f = c.fopen(str(p).encode(), b"rb")
    assert not L.BZ2_bzReadOpen(ctypes.byref(e), f, 0, 2, None, 0) and e.value == B.BZ_PARAM_ERROR  # small
    assert not L.BZ2_bzReadOpen(ctypes.byref(e), f, 0, 0, None, 3) and e.value == B.BZ_PARAM_ERROR  # unused
    assert not L.BZ2_bzWriteOpen(ctypes.byref(e), f, 10, 0, 30) and e.value == B.BZ_PARAM_ERROR  # level
    h = L.BZ2_bzReadOpen(ctypes.byref(e), f, 0, 0, None, 0)
    buf = ctypes.create_string_buffer(16)
    assert L.BZ2_bzRead(ctypes.byref(e), h, buf, 16) == 0 and e.value == B.BZ_UNEXPECTED_EOF  # empty file
    L.BZ2_bzReadGetUnused(ctypes.byref(e), h, ctypes.byref(ctypes.c_void_p()), ctypes.byref(ctypes.c_int()))
    assert e.value == B.BZ_SEQUENCE_ERROR  # only after STREAM_END
    L.BZ2_bzReadClose(ctypes.byref(e), h)
    c.fclose(f)


def test_randomised_block_streaming_decoder(lib, tmp_path):
    """BZ2_bzDecompress in small pieces and BZ2_bzRead decode a randomised block (the format's
    pre-0.9.5 random mask, bzlib.c:535-581) to the reference's output
    (tests/golden/randomised.bz2, made by tests/golden/make_randomised.py)."""
    from tests import oracles as O
    g = os.path.join(ROOT, "tests", "golden")
    comp = open(os.path.join(g, "randomised.bz2"), "rb").read()
    want = open(os.path.join(g, "randomised.out"), "rb").read()
    if O.has_ref():
        rc, ref_out = O.ref_decompress(comp, len(want) + 64)
        assert rc == 0 and ref_out == want
    strm = B.bz_stream()
    assert lib.BZ2_bzDecompressInit(ctypes.byref(strm), 0, 0) == 0
    inb = ctypes.create_string_buffer(comp, len(comp))
    ob = ctypes.create_string_buffer(1000)
    out, pos, rc = bytearray(), 0, 0
    while rc != B.BZ_STREAM_END:
        step = min(97, len(comp) - pos)
        strm.next_in = ctypes.cast(ctypes.byref(inb, pos), ctypes.c_void_p)
        strm.avail_in = step
        strm.next_out = ctypes.cast(ob, ctypes.c_void_p)
        strm.avail_out = 1000
        rc = lib.BZ2_bzDecompress(ctypes.byref(strm))
        assert rc in (0, B.BZ_STREAM_END), rc
        out += ob.raw[: 1000 - strm.avail_out]
        pos += step - strm.avail_in
    lib.BZ2_bzDecompressEnd(ctypes.byref(strm))
    assert bytes(out) == want
    assert B.buff_to_buff_decompress(comp, len(want) + 10) == want
    L = _file_api(lib)
    p = tmp_path / "r.bz2"
    p.write_bytes(comp)
    c = _libc()
    f = c.fopen(str(p).encode(), b"rb")
    e = ctypes.c_int(0)
    h = L.BZ2_bzReadOpen(ctypes.byref(e), f, 0, 0, None, 0)
    got = bytearray()
    big = ctypes.create_string_buffer(4096)
    while e.value == B.BZ_OK:
        n = L.BZ2_bzRead(ctypes.byref(e), h, big, 4096)
        got += big.raw[:n]
    assert e.value == B.BZ_STREAM_END and bytes(got) == want
    L.BZ2_bzReadClose(ctypes.byref(e), h)
    c.fclose(f)


def test_copy_rank_closed_forms_vs_reference(lib):
    """A5 on the device, section 8f row 4: the closed forms origptr.hip evaluates (one B* offset
    per period; several B* offsets in pairwise different (c0, c1) buckets within the reference's
    rank-stage budget, copyrank_cf.cpp) against the reference build, on random roots of every
    shape; the roots they leave go to the host model.  Also pins the share they cover."""
    from tests import datagen, oracles as O
    if not O.has_ref():
        pytest.skip("oracle/_ref not built")
    import random
    rng = random.Random(8402)
    txt = datagen.text(200_000, 21)
    multi = covered = checked = 0
    cases = [(b"hello world\n", k) for k in (2, 3, 8, 9, 10, 1024, 1025, 2049, 74_998)]
    cases += [(b"abac", k) for k in (2, 9, 17, 1000, 1025, 1026, 224_995)]
    cases += [(b"cab", k) for k in (2, 9, 1025)]  # (class q - 1 has the smallest bucket)
    for _ in range(1500):
        mode = rng.random()
        if mode < 0.5:
            w = bytes(rng.randrange(rng.choice([2, 3, 4, 8, 26, 256])) for _ in range(rng.randint(2, 16)))
        elif mode < 0.8:
            s = rng.randrange(0, len(txt) - 200)
            w = txt[s:s + rng.randint(4, 200)]
        else:
            w = bytes(rng.randrange(256) for _ in range(rng.randint(2, 40)))
        k = rng.choice([2, 3, 7, 9, 16, 100, 1023, 1024, 1025, 1026, 3000, rng.randint(2, 20000)])
        cases.append((w, k))
    for w, k in cases:
        if len(set(w)) < 2 or len(w) * k > 899_981:
            continue
        blk = w * k
        # primitive roots only
        p = len(w)
        if any(p % d == 0 and w == w[:d] * (p // d) for d in range(1, p)):
            continue
        r = B.copy_rank_closed_form(w, k)
        multi += 1
        if r < 0:
            continue
        covered += 1
        ref = O.ref_blocksort(blk)[1]
        rank = sum(1 for i in range(1, p) if (w[i:] + w[:i]) < w)
        assert rank * k + r == ref, (w[:24], k, r, ref)
        checked += 1
    assert checked >= 500 and covered / multi > 0.3, (checked, covered, multi)
