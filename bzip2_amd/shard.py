"""One .bz2 stream sharded across ranks: one process per GPU, each rank holding a
contiguous shard of the input in HBM; rank 0 ends up with the single stream that
BZ2_bzBuffToBuffCompress would have written for the whole input (bit-exact, any rank count).

Steps of `compress_sharded` (names follow the reference: blocks, runs, chunks, cuts):

1. Block cuts.  bzlib.c:211-315 copy_input_until_stop ends a block once it holds >= nblockMAX
   (100000*L - 19) RLE1 bytes; the pending run (a "chunk": <= 255 equal bytes) starts the next
   block, and in FINISH the last input byte never starts a block by itself (bzlib.c:276-308,
   361-396).  Cuts therefore depend on every byte before them and are walked rank after rank.
   Off the critical path each rank maps its shard's RLE1 chunks on the GPU (`bzg_seg_map`,
   from the shard's first run start); on it, a rank receives the open chunk and block fill at
   its shard start from the rank before, settles the run that crosses the boundary here on the
   host (arithmetic over 255-byte chunks), runs the device walk (`bzg_seg_walk`) and passes
   the open chunk at its shard end on.  One small message per rank.
2. Ownership.  All ranks all-gather the cuts.  A block belongs to the rank whose shard holds
   its first byte; a rank's range ends where the next owned block starts, so the bytes of its
   last block that lie in later shards come over point-to-point (xGMI).
3. Compression.  Each rank compresses its range with bzg_compress_device as a flushed segment
   (the range ends on a global cut, so its blocks equal the global ones): no header except
   on the owner of block 0, no trailer; the combined CRC starts from 0.
4. Gather.  An all-gather of {bits, blocks, combined CRC, first byte} gives each rank its bit
   offset; it shifts its bits to that offset mod 8 on the device and sends them to rank 0
   (the byte shared by two ranks is OR-merged there).  Rank 0 composes the combined CRC,
   combined = rotl(combined, blocks_r) ^ crc_r (compress.c:826-828), and appends the trailer
   (compress.c:863-869).

The GPU backend is the product path; tests inject a CPU stand-in backend (gloo, world size 2+).
"""
from __future__ import annotations

import ctypes
import time

import torch
import torch.distributed as dist

from . import BZG_FLAG_END_SEGMENT, BZG_FLAG_TAIL_MERGE, bound, bzg_stream_state, compress_device, lib, seg_map, \
    seg_walk

TRAILER_MAGIC = 0x177245385090
PIECE_MAX = 1_500_000_000  # bzg_seg_map region limit (32-bit RLE1 offsets)
# compress_sharded(..., timing=True): synchronise after each step and keep the host times
# (seconds since the call started) in last_timing (bench.py's phases_ms, outside its timed region)
_timing = False
last_timing: dict = {}
last_meta: dict = {}  # rank 0: blocks and payload bits of the last stream


def _mark(name: str, t0: float, dev) -> None:
    if _timing:
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        last_timing[name] = round(time.perf_counter() - t0, 6)


def nblock_max(level: int) -> int:
    return 100000 * level - 19


def chunk_size(length: int) -> int:
    """RLE1 bytes of one chunk of `length` equal bytes (bzlib.c:238-259 add_pair_to_block)."""
    return length if length < 4 else 5


def first_run_start(d: torch.Tensor) -> int:
    """Smallest j >= 1 with d[j] != d[j-1], or len(d)."""
    n = d.numel()
    w = 1 << 20
    lo = 1
    while lo < n:
        hi = min(n, lo + w)
        ne = d[lo:hi] != d[lo - 1:hi - 1]
        if bool(ne.any()):
            return lo + int(torch.argmax(ne.to(torch.uint8)))
        lo = hi
        w *= 4
    return n


def extend_run(t: int, fill: int, x: int, mx: int, cuts: list, last_pos: int):
    """Walk the chunks of a run piece [t, x) of equal bytes whose first chunk starts at t: chunks
    start every 255 bytes; each full chunk adds 5 RLE1 bytes and a chunk start is a cut once the
    block holds >= mx bytes (never at the stream's last byte, `last_pos`).  Returns the last
    chunk start (< x) and the fill there."""
    q = (x - t - 1) // 255  # chunk starts after t inside the piece
    while q > 0:
        need = max(1, -(-(mx - fill) // 5))
        if need <= q:
            t += 255 * need
            q -= need
            if t != last_pos:
                cuts.append(t)
                fill = 0
            else:
                fill += 5 * need
        else:
            t += 255 * q
            fill += 5 * q
            q = 0
    return t, fill


class GpuBackend:
    """The product path: bzg_seg_map / bzg_seg_walk / bzg_compress_device on the current device."""

    def __init__(self, level: int, stream_ptr: int = 0):
        self.level = level
        self.sp = stream_ptr

    def map_region(self, d: torch.Tensor) -> None:
        seg_map(d.data_ptr(), d.numel(), self.level, self.sp)

    def walk(self, fill: int, final: bool, n: int):
        # RLE1 can grow the input by 5/4 (runs of exactly 4 bytes): size the cut list as the
        # device sizes its own (rle1.hip seg_walk_stage: n + n/4 + 64 RLE1 bytes at most)
        return seg_walk(fill, final, (n + n // 4 + 64) // nblock_max(self.level) + 8)

    def compress(self, d: torch.Tensor, header: bool, final: bool):
        """Returns (bytes tensor holding `nbits` bits MSB-first, nbits, blocks, combined CRC)."""
        st = bzg_stream_state()
        lib().bzg_stream_init(ctypes.byref(st), self.level)
        st.header_done = 0 if header else 1
        cap = bound(d.numel()) + 16
        out = torch.empty(cap, dtype=torch.uint8, device=d.device)
        flags = BZG_FLAG_END_SEGMENT | (BZG_FLAG_TAIL_MERGE if final else 0)
        ob, cons, st = compress_device(d.data_ptr(), d.numel(), self.level, out.data_ptr(), cap, flags=flags,
                                       state=st, stream_ptr=self.sp)
        assert cons == d.numel()
        nbits = 8 * ob + st.carry_bits
        if st.carry_bits:
            out[ob] = st.carry_byte
        return out[:(nbits + 7) // 8], nbits, st.blocks_done, st.combined_crc


def piece_info(d: torch.Tensor):
    """(first byte, last byte, first run start) of a piece: device reads done before the chain."""
    return int(d[0]), int(d[-1]), first_run_start(d)


def chain_piece(be, d: torch.Tensor, s: int, n_total: int, msg, final: bool, mapped: bool = False, info=None):
    """Step 1 for one piece d = input[s, s + len(d)).  msg: None at the stream start, else the open
    chunk (t, fill, byte, covered) with t + covered == s.  `mapped`: bzg_seg_map already ran on
    d[first run start:]; `info`: piece_info(d) if already known.  Returns (global cuts, message
    on)."""
    mx = nblock_max(be.level)
    e = s + d.numel()
    last_pos = n_total - 1
    cuts: list = []
    d0, dlast, p = info if info is not None else piece_info(d)
    if msg is None:
        t, fill = s, 0
    else:
        t, fill, b, cov = msg
        if b != d0 or cov >= 255:  # the open chunk ends at s; a new one starts here
            fill += chunk_size(cov)
            t = s
            if fill >= mx and s != last_pos:
                cuts.append(s)
                fill = 0
    x = s + p  # [t, x) is one run piece of byte d0
    t, fill = extend_run(t, fill, x, mx, cuts, last_pos)
    if p == d.numel():
        return cuts, (None if final else (t, fill, d0, e - t))
    fill += chunk_size(x - t)  # the run ends at x, a run start
    if x == last_pos:  # the stream's last byte never opens a block: it joins the open one
        return cuts, None
    if fill >= mx:
        cuts.append(x)
        fill = 0
    if not mapped:
        be.map_region(d[p:])
    rc, lc, lf = be.walk(fill, final, d.numel() - p)
    cuts += [x + c for c in rc]
    if final:
        return cuts, None
    return cuts, (x + lc, lf, dlast, e - (x + lc))


def shift_bits(buf: torch.Tensor, nbits: int, sh: int) -> torch.Tensor:
    """buf's first nbits bits moved `sh` bits later (0 <= sh < 8); ceil((nbits + sh) / 8) bytes."""
    nb = (nbits + 7) // 8
    x = buf[:nb].clone()
    if nbits % 8:
        x[nb - 1] &= (0xFF << (8 - nbits % 8)) & 0xFF
    if sh == 0:
        return x
    out = torch.zeros(nb + 1, dtype=torch.uint8, device=buf.device)
    out[:nb] |= x >> sh
    out[1:] |= x << (8 - sh)
    return out[:(nbits + sh + 7) // 8]


def _dist_on() -> bool:
    return dist.is_available() and dist.is_initialized()


def _comm_dev(t: torch.Tensor) -> torch.Tensor:
    return t.cpu() if dist.get_backend() == "gloo" else t


def _all_gather_i64(vals, device):
    if not _dist_on():  # a single process: the stream is this shard
        return [list(vals)]
    t = torch.tensor(vals, dtype=torch.int64, device=device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def compress_sharded(d: torch.Tensor, shard_start: int, n_total: int, level: int, backend=None, timing: bool = False):
    """Compress input[shard_start, shard_start + len(d)) as this rank's shard of one stream of
    n_total bytes.  Every rank calls it (without a process group: one rank holding it all);
    rank 0 returns the whole .bz2 stream (a uint8 tensor on d's device, or on the CPU under
    gloo), the others None.  Shards are contiguous, in rank
    order and non-empty; n_total >= 1.  timing: record the phase times in last_timing."""
    global _timing
    _timing = timing
    be = backend or GpuBackend(level, torch.cuda.current_stream().cuda_stream if d.is_cuda else 0)
    t0 = time.perf_counter()
    last_timing.clear()
    rank, world = (dist.get_rank(), dist.get_world_size()) if _dist_on() else (0, 1)
    gloo = _dist_on() and dist.get_backend() == "gloo"
    cdev = "cpu" if gloo or not d.is_cuda else d.device
    n = d.numel()
    assert n > 0 and n_total > 0
    bounds = _all_gather_i64([shard_start, n], cdev)
    assert all(bounds[r][0] + bounds[r][1] == bounds[r + 1][0] for r in range(world - 1))
    assert bounds[0][0] == 0 and bounds[-1][0] + bounds[-1][1] == n_total

    # 1. block cuts, rank after rank
    pieces = [(o, min(PIECE_MAX, n - o)) for o in range(0, n, PIECE_MAX)]
    info0 = piece_info(d[:pieces[0][1]])  # device reads off the chain's critical path
    first_p = info0[2]
    if first_p < pieces[0][1]:
        be.map_region(d[first_p:pieces[0][1]])  # off the critical path
    _mark("map", t0, d.device)
    msg = None
    if rank > 0:
        m = torch.empty(5, dtype=torch.int64, device=cdev)
        dist.recv(m, rank - 1)
        ml = m.tolist()
        msg = None if ml[4] == 0 else tuple(ml[:4])
    cuts: list = []
    last_rank = rank == world - 1
    for i, (o, ln) in enumerate(pieces):
        c, msg = chain_piece(be, d[o:o + ln], shard_start + o, n_total, msg,
                             final=last_rank and i == len(pieces) - 1, mapped=(i == 0 and first_p < ln),
                             info=info0 if i == 0 else None)
        cuts += c
    if not last_rank:
        m = torch.tensor(list(msg) + [1], dtype=torch.int64, device=cdev)
        dist.send(m, rank + 1)
    _mark("chain", t0, d.device)

    # 2. ownership and the bytes of each rank's range that live in later shards
    cnt = _all_gather_i64([len(cuts)], cdev)
    mxc = max(c[0] for c in cnt)
    allc = _all_gather_i64(cuts + [-1] * (mxc - len(cuts)) if mxc else [-1], cdev)
    starts = [0] + [c for r in range(world) for c in allc[r][:cnt[r][0]]]
    owner_first = []
    for r in range(world):
        lo, hi = bounds[r][0], bounds[r][0] + bounds[r][1]
        owned = [b for b in starts if lo <= b < hi]
        owner_first.append(owned[0] if owned else None)
    ranges = []
    for r in range(world):
        if owner_first[r] is None:
            ranges.append((0, 0))
            continue
        nxt = next((owner_first[j] for j in range(r + 1, world) if owner_first[j] is not None), n_total)
        ranges.append((owner_first[r], nxt))
    lo, hi = ranges[rank]
    ops = []
    buf = None
    if hi > lo:
        own_hi = min(hi, shard_start + n)
        if hi <= shard_start + n:
            buf = d[lo - shard_start:hi - shard_start]
        else:
            buf = torch.empty(hi - lo, dtype=torch.uint8, device=d.device)
            buf[:own_hi - lo].copy_(d[lo - shard_start:own_hi - shard_start])
    recv_fix = []
    for r in range(world):  # r needs [max(lo_r, s_j), min(hi_r, e_j)) from every later shard j
        rlo, rhi = ranges[r]
        for j in range(r + 1, world):
            a, b = max(rlo, bounds[j][0]), min(rhi, bounds[j][0] + bounds[j][1])
            if a >= b:
                continue
            if rank == j:
                ops.append(dist.P2POp(dist.isend, _comm_dev(d[a - shard_start:b - shard_start].contiguous()), r))
            elif rank == r:
                tgt = buf[a - lo:b - lo]
                tmp = tgt if cdev == tgt.device else torch.empty(b - a, dtype=torch.uint8, device=cdev)
                ops.append(dist.P2POp(dist.irecv, tmp, j))
                if tmp is not tgt:
                    recv_fix.append((tgt, tmp))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    for tgt, tmp in recv_fix:
        tgt.copy_(tmp)

    _mark("halo", t0, d.device)

    # 3. compress the range
    if buf is not None:
        bits, nbits, nblk, crc = be.compress(buf, header=(lo == 0), final=(hi == n_total))
    else:
        bits, nbits, nblk, crc = torch.zeros(1, dtype=torch.uint8, device=d.device), 0, 0, 0

    _mark("compress", t0, d.device)

    # 4. bit offsets, shift, gather to rank 0, trailer
    meta0 = _all_gather_i64([nbits, nblk, crc], cdev)
    off = sum(meta0[r][0] for r in range(rank))
    total_bits = sum(m[0] for m in meta0)
    sh = off % 8
    y = shift_bits(bits, nbits, sh) if nbits else torch.zeros(1, dtype=torch.uint8, device=d.device)
    meta = _all_gather_i64([int(y[0]) if nbits else 0], cdev)
    out_len = (total_bits + 80 + 7) // 8
    ops = []
    final = None
    if rank == 0:
        final = torch.zeros(out_len, dtype=torch.uint8, device=cdev)
        if nbits:
            final[:y.numel()].copy_(y)
        o = 0
        for r in range(world):
            nb_r = meta0[r][0]
            if r > 0 and nb_r:
                ln = ((o % 8) + nb_r + 7) // 8
                if ln > 1:
                    ops.append(dist.P2POp(dist.irecv, final[o // 8 + 1:o // 8 + ln], r))
            o += nb_r
    elif nbits and y.numel() > 1:
        ops.append(dist.P2POp(dist.isend, _comm_dev(y[1:].contiguous()), 0))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    _mark("gather", t0, d.device)
    if rank != 0:
        return None
    o = 0
    for r in range(world):
        if r > 0 and meta0[r][0]:
            final[o // 8] |= meta[r][0]
        o += meta0[r][0]
    combined = 0
    for r in range(world):
        k = meta0[r][1] % 32
        combined = (((combined << k) | (combined >> (32 - k))) & 0xFFFFFFFF) if k else combined
        combined ^= meta0[r][2]
    last_meta.update(blocks=sum(m[1] for m in meta0), bits=total_bits, combined_crc=combined)
    tr = ((TRAILER_MAGIC << 32) | combined).to_bytes(10, "big")
    tt = shift_bits(torch.tensor(list(tr), dtype=torch.uint8, device=cdev), 80, total_bits % 8)
    base = total_bits // 8
    final[base] |= tt[0]
    final[base + 1:base + tt.numel()] = tt[1:]
    _mark("trailer", t0, d.device)
    return final
