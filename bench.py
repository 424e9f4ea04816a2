"""bench.py -- input-side MB/s of the MI355X bzip2 compression path at -9 (BASELINE.json metric).

Workload (per GPU): 1e9 bytes of seeded enwik9-class synthetic text (tests/datagen.py; enwik9
itself is not available offline), resident in HBM before the timed region; one step = one
complete .bz2 stream (RLE1 -> BWT -> MTF -> Huffman -> packing, bit-exact with the reference)
written to HBM.  N GPUs = N ranks, each compressing its own 1e9-byte stream (independent
objects, no data-path collective): scaling "weak", value = total bytes / max-over-ranks time.
`--gpus N` with N > 1 and no WORLD_SIZE in the environment launches the N ranks itself (a child
`torch.distributed.run` on 127.0.0.1, started before this process touches the GPU); under an
outside launcher the world size must equal `--gpus`.

Also reported on rank 0: the reference CPU path timed on a bounded sample of the same text
(oracle/_ref = the reference's own blocksort.c/compress.c build, 1 thread), a bit-exactness
check of the GPU stream against it on that sample, the per-stage split from HIP events, and
the roofline of SURVEY.md section 8(d): B_alg = 1 + 25*rho + 3*c bytes per input byte against
the 8 TB/s HBM peak.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bzip2_amd as B  # noqa: E402
from tests import datagen  # noqa: E402

METRIC = "input-side MB/s at -9 on enwik9, bit-exact .bz2, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--bytes", type=int, default=1_000_000_000, help="input bytes per GPU (weak scaling)")
    p.add_argument("--total-bytes", type=int, default=0,
                   help="strong scaling: ONE stream of this many bytes split into N contiguous shards, one per "
                        "rank (BASELINE config 3: --total-bytes 1000000000); implies --mode stream")
    p.add_argument("--level", type=int, default=9)
    p.add_argument("--cpu-sample", type=int, default=300_000_000, help="bytes for the CPU reference timing")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=16,
                   help="threads for the multi-core reference baseline (the box's CPU share is 16)")
    p.add_argument("--cpu-mt-sample", type=int, default=640_000_000, help="bytes for the multi-core timing")
    p.add_argument("--no-h2h", action="store_true", help="skip the host-to-host region (profiling runs)")
    p.add_argument("--repeat-frac", type=float, default=0.0,
                   help="overwrite this fraction of the text with copies of earlier passages (profiling the "
                        "long-repeat path; the default workload has none)")
    p.add_argument("--no-extra", action="store_true",
                   help="skip the secondary lines (BASELINE configs 4 and 5, long-repeat text)")
    p.add_argument("--mode", choices=["stream", "independent"], default=None,
                   help="stream: the ranks' inputs are consecutive shards of ONE .bz2 stream, gathered on "
                        "rank 0 (bzip2_amd/shard.py; default for N > 1); independent: one stream per rank")
    return p.parse_args()


def max_over_ranks(x: float, device) -> float:
    """The job's time: the maximum of the ranks' timed regions (all_reduce MAX)."""
    t = torch.tensor([x], dtype=torch.float64, device=device)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def job_mbps(bytes_per_rank: int, world: int, steps: int, elapsed: float) -> float:
    """Whole-job input-side MB/s: every rank's bytes over the slowest rank's time."""
    return bytes_per_rank * world * steps / elapsed / 1e6


def rank_seed(rank: int) -> int:
    """Each rank compresses its own synthetic object (weak scaling, no shared input)."""
    return 0x5EED0001 + rank


def shard_bounds(total: int, world: int, rank: int) -> tuple:
    """Strong scaling: rank r holds input[total * r // world, total * (r + 1) // world) of the one
    job input (contiguous, in rank order, sizes differing by at most one byte)."""
    return total * rank // world, total * (rank + 1) // world


def job_layout(a, world: int, rank: int) -> dict:
    """What this rank compresses.  Weak (default): its own a.bytes (one shard of a stream of world x
    a.bytes bytes in stream mode, or an independent stream).  Strong (--total-bytes T): shard
    `rank` of ONE stream of T bytes (BASELINE config 3 at T = 1e9)."""
    if a.total_bytes:
        lo, hi = shard_bounds(a.total_bytes, world, rank)
        return {"scaling": "strong", "mode": "stream", "lo": lo, "n": hi - lo, "job_bytes": a.total_bytes,
                "seed": rank_seed(0)}
    mode = a.mode or ("stream" if world > 1 else "independent")
    return {"scaling": "weak", "mode": mode, "lo": rank * a.bytes, "n": a.bytes, "job_bytes": world * a.bytes,
            "seed": rank_seed(rank)}


def launch_cmd(argv, n: int, port: int) -> list:
    """The child command that runs this bench as n ranks of one node (one process per GPU)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a, argv) -> int:
    """`--gpus N` (N > 1) without an outside launcher: run N ranks as a child process group and
    return its exit code.  Nothing in this process has touched the GPU yet (no exec either)."""
    import subprocess

    if os.environ.get("BZG_DIST_BACKEND") != "gloo":
        have = torch.cuda.device_count()  # does not initialise the GPU on this image
        if have < a.gpus:
            print(f"bench.py: --gpus {a.gpus} but {have} GPU(s) visible (BZG_DIST_BACKEND=gloo rehearses "
                  f"several ranks on one GPU)", file=sys.stderr)
            return 2
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(launch_cmd(argv, a.gpus, free_port()), env=env).returncode


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print(f"bench.py: world size {world} != --gpus {a.gpus}", file=sys.stderr)
        sys.exit(2)
    if os.environ.get("BZG_BENCH_PROBE") == "1":  # launcher test (CPU): report the rank layout only
        r = int(os.environ.get("RANK", "0"))
        probe = {"rank": r, "world": world, "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                 "master": os.environ.get("MASTER_ADDR")}
        if a.total_bytes:
            lay = job_layout(a, world, r)
            probe.update(scaling=lay["scaling"], mode=lay["mode"], lo=lay["lo"], n=lay["n"], job_bytes=lay["job_bytes"])
        print(json.dumps(probe), flush=True)
        return
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if os.environ.get("BZG_DIST_BACKEND") == "gloo":  # rehearsal: every rank on the box's one GPU
        local = 0
    torch.cuda.set_device(local)
    lay = job_layout(a, world, rank)
    mode = lay["mode"]
    strong = lay["scaling"] == "strong"
    if dist:
        backend = os.environ.get("BZG_DIST_BACKEND", "nccl")  # gloo: multi-rank rehearsal on one GPU
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group(backend)

    t0 = time.time()
    if strong:  # every rank makes the one job input and keeps its shard
        data = datagen.text(a.total_bytes, lay["seed"])[lay["lo"]:lay["lo"] + lay["n"]]
    else:
        data = datagen.text(a.bytes, lay["seed"])
    gen_s = time.time() - t0
    d_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda")
    if a.repeat_frac > 0:
        add_repeats(d_in, a.repeat_frac)
        data = d_in.cpu().numpy().tobytes()
    cap = B.bound(len(data))
    d_out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream

    last_stream = [None]

    def step():
        if mode == "stream":
            from bzip2_amd import shard

            res = shard.compress_sharded(d_in, lay["lo"], lay["job_bytes"], a.level)
            last_stream[0] = res
            return res.numel() / world if res is not None else 0  # per-rank share of the one stream
        nb, cons, _ = B.compress_device(d_in.data_ptr(), len(data), a.level, d_out.data_ptr(), cap, stream_ptr=sp)
        return nb

    for _ in range(a.warmup):
        out_bytes = step()
    torch.cuda.synchronize()
    stage_ms = {"rle1": 0.0, "bwt": 0.0, "mtf": 0.0, "code": 0.0, "total": 0.0}
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(a.steps):
        out_bytes = step()
        s = B.last_stats()
        for k in ("rle1", "bwt", "mtf", "code", "total"):
            stage_ms[k] += s[k + "_ms"] / a.steps
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t_start
    if dist:
        elapsed = max_over_ranks(elapsed, "cuda")
    stats = B.last_stats()
    ms_per_step = elapsed * 1000.0 / a.steps
    value = lay["job_bytes"] * a.steps / elapsed / 1e6  # MB/s, whole job (= job_mbps(a.bytes, world, ...) when weak)
    phases = None
    if mode == "stream":  # one more step, untimed, with a synchronisation after each phase
        from bzip2_amd import shard

        shard.compress_sharded(d_in, lay["lo"], lay["job_bytes"], a.level, timing=True)
        tm = dict(shard.last_timing)
        prev, phases = 0.0, {}
        for k in ("map", "chain", "halo", "compress", "gather", "trailer"):
            if k in tm:
                phases[k] = round((tm[k] - prev) * 1e3, 3)
                prev = tm[k]
        if dist:
            allp = [None] * world
            torch.distributed.all_gather_object(allp, phases)
            phases = {"rank%d" % r: p for r, p in enumerate(allp)}

    if mode == "stream" and rank != 0:
        stream_parity(None, d_in, a, world)  # sends this rank's shard to rank 0
        stream_ref_check(d_in, a, world)
    if rank == 0:
        nbytes = lay["n"] if not (mode == "stream") else lay["job_bytes"] / world  # per-rank share
        ratio = out_bytes / nbytes
        rho = stats["rle_bytes"] / lay["n"]
        b_alg = 1.0 + 25.0 * rho + 3.0 * ratio
        achieved = lay["job_bytes"] / world * b_alg / (ms_per_step / 1000.0) / 1e9
        bwt_alg = 11.0 * stats["rle_bytes"]  # read T + write SA + read SA + gather T + write L
        result = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "MB/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": lay["scaling"],
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": (f"BASELINE config 3: enwik9-class synthetic text (tests/datagen.py), ONE stream of "
                                    f"{a.total_bytes} B split over {world} rank(s), -{a.level}") if strong else
                                   f"enwik9-class synthetic text (tests/datagen.py), {a.bytes} B per GPU, -{a.level}",
                       "level": a.level, "bytes_per_gpu": lay["n"], "job_bytes": lay["job_bytes"],
                       "blocks": stats["nblocks"],
                       "bz2_ratio": round(ratio, 4), "rle1_rho": round(rho, 4),
                       "parallelism": (f"one stream of {lay['job_bytes']} B sharded over {world} ranks "
                                       "(RCCL cut chain, P2P halo, bitstream gather to rank 0)")
                       if mode == "stream" else f"{world} independent streams"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 5), "traffic": None,
                         "traffic_note": "no PMC profile for this workload under profiles/",
                         "model": "SURVEY.md 8(d) B_alg = 1 + 25*rho + 3*c bytes per input byte, whole pipeline",
                         "b_alg_per_byte": round(b_alg, 3),
                         "dominant_stage": {"name": "bwt", "ms": round(stage_ms["bwt"], 3),
                                            "alg_bytes": bwt_alg,
                                            "achieved_GBps": round(bwt_alg / (stage_ms["bwt"] / 1e3) / 1e9, 2)
                                            if stage_ms["bwt"] > 0 else None}},
            "stages_ms": {k: round(v, 3) for k, v in stage_ms.items()},
            "sort_iterations": stats["sort_iterations"],
            **({"phases_ms": phases, "phases_note": "one extra untimed step synchronised after each phase of "
                                                     "compress_sharded (bzip2_amd/shard.py)"} if phases else {}),
            "gen_s": round(gen_s, 1),
        }
        if mode == "stream" and last_stream[0] is not None:
            result["stream_check"] = stream_parity(last_stream[0], d_in, a, world)
            result["stream_check"]["reference"] = stream_ref_check(d_in, a, world)
        pmc = pmc_traffic(a) if not strong and mode == "independent" else None
        if pmc is not None:
            rl = result["roofline"]
            rl["traffic"] = round(pmc["traffic_B_per_step"] / (ms_per_step / 1e3) / 1e9, 2)
            rl["traffic_note"] = (f"GB/s: HBM bytes per step from rocprofv3 FETCH_SIZE/WRITE_SIZE passes of this "
                                  f"workload ({pmc['file']}, {pmc['correction']}; uncorrected "
                                  f"{pmc['traffic_lower_B_per_step'] / 1e9:.1f} GB) over this run's step time")
            rl["traffic_B_per_step"] = round(pmc["traffic_B_per_step"])
        if not a.no_h2h and not strong:
            result["host_to_host"] = host_to_host(data, a, cap)
        if not a.no_cpu:
            result.update(cpu_and_parity(data, a, d_in))
        if not a.no_extra and mode == "independent":
            result["secondary"] = extra_configs(a, d_in, d_out, cap, no_cpu=a.no_cpu, nb_text=out_bytes)
        print(json.dumps(result), flush=True)
    if dist:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


def stream_parity(stream, d_in, a, world):
    """Outside the timed region: the sharded stream must equal, byte for byte, the plain
    single-device bzg_compress_device call over the whole input (all shards gathered on rank 0),
    i.e. the output does not depend on the rank count (SURVEY.md 4.3 determinism)."""
    import torch.distributed as dist

    rank = dist.get_rank() if world > 1 else 0
    gloo = world > 1 and dist.get_backend() == "gloo"
    if rank != 0:
        dist.send(d_in.cpu() if gloo else d_in, 0)
        return None
    lays = [job_layout(a, world, r) for r in range(world)]
    total = lays[0]["job_bytes"]
    full = torch.empty(total, dtype=torch.uint8, device="cuda")
    full[:lays[0]["n"]].copy_(d_in)
    for r in range(1, world):
        lo, n = lays[r]["lo"], lays[r]["n"]
        if gloo:
            tmp = torch.empty(n, dtype=torch.uint8)
            dist.recv(tmp, r)
            full[lo:lo + n].copy_(tmp)
        else:
            dist.recv(full[lo:lo + n], r)
    cap = B.bound(total)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    nb, _, _ = B.compress_device(full.data_ptr(), total, a.level, out.data_ptr(), cap)
    torch.cuda.synchronize()
    s = stream.to("cuda")
    eq = nb == s.numel() and bool(torch.equal(out[:nb], s))
    del full, out
    torch.cuda.empty_cache()
    return {"bytes": int(s.numel()), "ranks": world, "equals_single_device_stream": eq,
            "against": f"bzg_compress_device over all {total} B on one device"}


def stream_ref_check(d_in, a, world, per_rank: int = 3_000_000):
    """Outside the timed region, every rank: the first per_rank bytes of each rank's shard form
    one sample stream compressed by the same sharded path (cut chain, halo, gather over the
    job's backend), with a shard boundary every per_rank bytes; rank 0 compares it byte for
    byte with the reference build (oracle/_ref) on the concatenated sample."""
    import torch.distributed as dist
    from bzip2_amd import shard

    rank = dist.get_rank() if world > 1 else 0
    gloo = world > 1 and dist.get_backend() == "gloo"
    k = min(per_rank, min(job_layout(a, world, r)["n"] for r in range(world)))  # the same on every rank
    piece = d_in[:k].contiguous()
    res = shard.compress_sharded(piece, rank * k, world * k, a.level)
    if rank != 0:
        dist.send(piece.cpu() if gloo else piece, 0)
        return None
    parts = [piece.cpu()]
    for r in range(1, world):
        tmp = torch.empty(k, dtype=torch.uint8, device="cpu" if gloo else "cuda")
        dist.recv(tmp, r)
        parts.append(tmp.cpu())
    sample = torch.cat(parts).numpy().tobytes()
    from tests import oracles as O

    if not O.has_ref():
        return {"sample_bytes": len(sample), "ranks": world, "bit_exact": None, "against": "oracle/_ref absent"}
    want = O.ref_compress(sample, a.level)
    got = res.cpu().numpy().tobytes()
    return {"sample_bytes": len(sample), "ranks": world, "shard_bytes": k, "bit_exact": got == want,
            "against": "reference (oracle/_ref BZ2_bzBuffToBuffCompress on the concatenated sample)"}


def time_device(d, n, level, d_out, cap, steps, warmup=1):
    """ms per call of bzg_compress_device on n device-resident bytes, and the last stats."""
    sp = torch.cuda.current_stream().cuda_stream
    for _ in range(warmup):
        nb, _, _ = B.compress_device(d.data_ptr(), n, level, d_out.data_ptr(), cap, stream_ptr=sp)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        nb, _, _ = B.compress_device(d.data_ptr(), n, level, d_out.data_ptr(), cap, stream_ptr=sp)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3 / steps, nb, B.last_stats()


def sequential_stages(d, n, level, d_out, cap):
    """A multi-batch input's stage split with its batches one after another (one untimed step,
    BZG_BATCH_PIPE=0): the pipelined run's stage figures are per-batch event spans that overlap
    (a batch's MTF / tables / packing beside the next batch's sorts), so their sum exceeds the
    step time."""
    os.environ["BZG_BATCH_PIPE"] = "0"
    try:
        ms, _, st = time_device(d, n, level, d_out, cap, steps=1, warmup=0)
    finally:
        del os.environ["BZG_BATCH_PIPE"]
    return {"ms": round(ms, 3), "stages_ms": {k: round(st[k + "_ms"], 3) for k in ("rle1", "bwt", "mtf", "code")},
            "note": "one step with the batches one after another (BZG_BATCH_PIPE=0); stages_ms of the pipelined "
                    "line above are overlapping per-batch spans"}


def line_for(name, n, level, ms, nb, st, workload):
    rho = st["rle_bytes"] / n
    c = nb / n
    b_alg = 1.0 + 25.0 * rho + 3.0 * c
    return {"workload": workload, "bytes": n, "level": level, "value": round(n / ms / 1e3, 2), "unit": "MB/s",
            "ms_per_step": round(ms, 3), "bz2_ratio": round(c, 5), "rle1_rho": round(rho, 5),
            "blocks": st["nblocks"], "sort_unsorted": st["sort_unsorted"],
            "stages_ms": {k: round(st[k + "_ms"], 3) for k in ("rle1", "bwt", "mtf", "code")},
            "roofline": {"bound": "hbm", "b_alg_per_byte": round(b_alg, 4),
                         "achieved": round(n * b_alg / (ms / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(n * b_alg / (ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 5)}}


def sample_parity(d, n, level, no_cpu):
    """GPU stream of d[:n] against the reference's (pinned child, timed) -> dict."""
    from tests import oracles as O

    cap = B.bound(n)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    nb, _, _ = B.compress_device(d.data_ptr(), n, level, out.data_ptr(), cap)
    torch.cuda.synchronize()
    got = out[:nb].cpu().numpy().tobytes()
    if no_cpu or not O.has_ref():
        return {"sample_bytes": n, "bit_exact": got == O.orc_compress(d[:n].cpu().numpy().tobytes(), level),
                "against": "port"}
    cpu_s, ref = run_cpu_child(d[:n].cpu().numpy().tobytes(), level, sorted(os.sched_getaffinity(0))[:1])
    return {"sample_bytes": n, "bit_exact": got == ref, "against": "reference",
            "cpu_baseline": {"value": round(n / cpu_s / 1e6, 3), "unit": "MB/s", "cores": 1, "kind": "reference",
                             "sample": f"first {n} B, BZ2_bzBuffToBuffCompress -{level}, pinned child"}}


def add_repeats(d, frac: float, seed: int = 0x5EED0009) -> None:
    """Overwrites about frac of d (in place, on the device) with copies of earlier passages of
    2 kB .. 200 kB: enwik-like long repeats (templates, reverted revisions)."""
    import random

    n = d.numel()
    rng = random.Random(seed)
    covered = 0
    while covered < int(n * frac):
        ln = rng.randint(2_000, 200_000)
        dst = rng.randrange(1_000_000, n - ln)
        src = rng.randrange(0, dst - ln) if rng.random() < 0.5 else max(0, dst - rng.randint(ln, 4 * ln))
        d[dst:dst + ln] = d[src:src + ln].clone()
        covered += ln


def decode_line(a, d_text, d_stream, nb, no_cpu):
    """GPU decompression of the main workload's stream, device resident:
    output-side MB/s, the output compared with the input, the reference decoder timed on a
    bounded sample in a pinned child.  Decode bytes model: read c + 18 rho + write 1 per output
    byte (L written 1, read twice 2, Q written 4 and read by two walks 8, Y written 1 and read
    twice 2)."""
    n = d_text.numel()
    d_dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    rc, got = B.decompress_device(d_stream.data_ptr(), nb, d_dec.data_ptr(), n + 64, stream_ptr=sp)
    torch.cuda.synchronize()
    ok = rc == 0 and got == n and bool(torch.equal(d_dec[:n], d_text))
    steps = 3
    t = time.perf_counter()
    for _ in range(steps):
        B.decompress_device(d_stream.data_ptr(), nb, d_dec.data_ptr(), n + 64, stream_ptr=sp)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3 / steps
    st = B.last_decode_stats()
    c = nb / n
    b_alg = c + 18.0 + 1.0
    line = {"workload": f"decompression of the main workload's -{a.level} stream ({nb} B -> {n} B), device resident",
            "bytes_out": n, "value": round(n / ms / 1e3, 2), "unit": "MB/s (output side)", "ms_per_step": round(ms, 3),
            "blocks": st["blocks"], "candidates": st["candidates"], "output_equals_input": ok,
            "roofline": {"bound": "hbm", "b_alg_per_byte": round(b_alg, 3),
                         "achieved": round(n * b_alg / (ms / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(n * b_alg / (ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 5)}}
    del d_dec
    from tests import oracles as O

    if not no_cpu and O.has_ref():
        m = 100_000_000
        sample = O.ref_compress(d_text[:m].cpu().numpy().tobytes(), a.level)
        secs, _ = run_cpu_child(sample, a.level, sorted(os.sched_getaffinity(0))[:1], op="d", cap=m)
        line["cpu_baseline"] = {"value": round(m / secs / 1e6, 3), "unit": "MB/s (output side)", "cores": 1,
                                "kind": "reference",
                                "sample": f"BZ2_bzBuffToBuffDecompress of the -{a.level} stream of the first {m} B, "
                                          f"pinned child"}
    return line


def small_call_lines(a, d_text, d_out, cap, no_cpu):
    """BASELINE config 2 (enwik8: 1e8 B of the same text generator, -9, one MI355X, device
    resident), bit-exact against the reference on the whole 100 MB; and the per-rank share of
    BASELINE config 3 at N = 2, 4, 8 (one call on 500, 250, 125 MB of the config-3 input: the
    compress phase of one rank under strong scaling), with the per-byte rate against 1 GB."""
    res = {}
    n2 = 100_000_000
    ms, nb, st = time_device(d_text, n2, a.level, d_out, cap, steps=10, warmup=2)
    line = line_for("enwik8", n2, a.level, ms, nb, st,
                    f"BASELINE config 2: the first {n2} B of the enwik9-class synthetic text (tests/datagen.py "
                    f"stands in for enwik8), -{a.level}, device resident")
    line["parity"] = sample_parity(d_text, n2, a.level, no_cpu)
    res["enwik8_100mb"] = line
    shares = {}
    t1g = None
    for n in (1_000_000_000, 500_000_000, 250_000_000, 125_000_000):
        if n > d_text.numel():
            continue
        ms, nb, st = time_device(d_text, n, a.level, d_out, cap, steps=5 if n >= 500_000_000 else 10, warmup=1)
        if n == 1_000_000_000:
            t1g = ms
        shares[str(n)] = {"ms": round(ms, 3), "value": round(n / ms / 1e3, 2), "unit": "MB/s",
                          "stages_ms": {k: round(st[k + "_ms"], 3) for k in ("rle1", "bwt", "mtf", "code")},
                          **({"ms_per_gb_vs_1gb": round(ms * (1e9 / n) / t1g, 3)} if t1g else {})}
    res["strong_shares"] = {"workload": "one bzg_compress_device call on the first n B of the config-3 input "
                                        "(the compress phase of one rank of a strong-scaling run at N = 1e9 / n)",
                            "shares": shares}
    return res


def extra_configs(a, d_text, d_out_text, cap_text, no_cpu=False, nb_text=0):
    """Secondary lines (never `value`): GPU decompression of the main stream, BASELINE configs 4
    and 5 at full size (4 GiB, device resident; bzg_compress_device cuts them into 1.5e9-byte
    batches), and enwik-like text with long duplicated passages (the sorter's deep-group path)."""
    res = {}
    if nb_text:
        res["decompress_text"] = decode_line(a, d_text, d_out_text, nb_text, no_cpu)
    # (after the decode line: these calls overwrite the main stream in d_out_text)
    res.update(small_call_lines(a, d_text, d_out_text, cap_text, no_cpu))
    n4 = 1 << 32
    level = 9
    d = torch.full((n4,), 0x61, dtype=torch.uint8, device="cuda")
    cap = B.bound(n4)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    ms, nb, st = time_device(d, n4, level, out, cap, steps=2)
    res["single_byte_4gib"] = line_for("single", n4, level, ms, nb, st, "4 GiB of byte 0x61 (BASELINE config 4), -9")
    res["single_byte_4gib"]["sequential"] = sequential_stages(d, n4, level, out, cap)
    res["single_byte_4gib"]["parity"] = sample_parity(d, 256 << 20, level, no_cpu)
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED0005)
    d = torch.randint(0, 256, (n4,), dtype=torch.uint8, device="cuda", generator=g)
    ms, nb, st = time_device(d, n4, level, out, cap, steps=2)
    res["random_4gib"] = line_for("random", n4, level, ms, nb, st,
                                  "4 GiB of seeded PRNG bytes (torch Philox, seed 0x5EED0005; BASELINE config 5), -9")
    res["random_4gib"]["sequential"] = sequential_stages(d, n4, level, out, cap)
    res["random_4gib"]["parity"] = sample_parity(d, 32 << 20, level, no_cpu)
    del d, out
    torch.cuda.empty_cache()
    # long repeats: 25% of the text overwritten by copies of earlier passages (2 kB .. 200 kB)
    n = d_text.numel()
    dr = d_text.clone()
    add_repeats(dr, 0.25)
    ms, nb, st = time_device(dr, n, level, d_out_text, cap_text, steps=2)
    res["long_repeat_text"] = line_for("long_repeat", n, level, ms, nb, st,
                                       f"the main workload with 25% overwritten by copies of earlier passages "
                                       f"(2-200 kB), {n} B, -9")
    res["long_repeat_text"]["parity"] = sample_parity(dr, 64 << 20, level, no_cpu)
    del dr
    torch.cuda.empty_cache()
    return res


def pmc_traffic(a):
    """HBM bytes per step of this workload, from the newest committed PMC summary
    (profiles/*_hbm_traffic_v*.json, written by tools/traffic.py); None if there is none."""
    import glob
    import re

    best = None
    for f in glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "*_hbm_traffic_v*.json")):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("bytes_per_step") != a.bytes or f"-{a.level}" not in d.get("workload", ""):
            continue
        v = int(re.search(r"_v(\d+)\.json$", f).group(1))
        if best is None or v > best[0]:
            d["file"] = "profiles/" + os.path.basename(f)
            best = (v, d)
    return best[1] if best else None


def host_to_host(data, a, cap):
    """SURVEY.md 8(d) second timed region: host buffers in and out (H2D + kernels + D2H),
    through BZ2_bzBuffToBuffCompress; never `value`."""
    import numpy as np
    src = np.frombuffer(data, dtype=np.uint8)
    dst = np.empty(cap, dtype=np.uint8)
    dl = ctypes.c_uint(cap)
    L = B.lib()

    def h2h_call():
        dl.value = cap
        rc = L.BZ2_bzBuffToBuffCompress(dst.ctypes.data, ctypes.byref(dl), src.ctypes.data, len(data),
                                        a.level, 0, 30)
        assert rc == B.BZ_OK, rc

    h2h_call()  # warm-up (host staging buffers)
    times = []
    for _ in range(3):  # one call is ~60 ms; PCIe and host-copy timing varies from call to call
        t1 = time.perf_counter()
        h2h_call()
        times.append(time.perf_counter() - t1)
    h2h = min(times)
    return {"value": round(a.bytes / h2h / 1e6, 2), "unit": "MB/s", "ms": round(h2h * 1e3, 3),
            "ms_calls": [round(t * 1e3, 3) for t in times], "out_bytes": int(dl.value),
            "api": "BZ2_bzBuffToBuffCompress, pageable host buffers (H2D + kernels + D2H), best of 3 warm calls"}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_child(path: str, level: int, cpus: str, op: str = "c", cap: int = 0) -> None:
    """`bench.py --cpu-child`: the reference CPU path (oracle/_ref, the reference's own
    blocksort.c/compress.c build) timed in a child process pinned to `cpus` (no GPU touched).
    One cpu: one BZ2_bzBuffToBuffCompress of the whole sample, output kept beside it for the
    parity check; k cpus: k threads, each compressing a contiguous 1/k of the sample as its own
    stream."""
    from concurrent.futures import ThreadPoolExecutor

    from tests import oracles as O

    cs = sorted(int(c) for c in cpus.split(","))
    os.sched_setaffinity(0, cs)
    data = open(path, "rb").read()
    nt = len(cs)
    if op == "d":  # the reference decoder on one .bz2 stream
        t = time.perf_counter()
        rc, out = O.ref_decompress(data, cap)
        dt = time.perf_counter() - t
        assert rc == 0 and len(out) == cap, rc
    elif nt == 1:
        t = time.perf_counter()
        out = O.ref_compress(data, level)
        dt = time.perf_counter() - t
        open(path + ".ref", "wb").write(out)
    else:
        step = -(-len(data) // nt)
        shards = [data[i:i + step] for i in range(0, len(data), step)]
        with ThreadPoolExecutor(nt) as ex:
            t = time.perf_counter()
            list(ex.map(lambda x: O.ref_compress(x, level), shards))
            dt = time.perf_counter() - t
    print(json.dumps({"seconds": dt, "bytes": len(data), "threads": nt}), flush=True)


def run_cpu_child(sample: bytes, level: int, cpus, op: str = "c", cap: int = 0) -> tuple:
    """Times the reference on `sample` in a pinned child (taskset when present); returns
    (seconds, reference output or None)."""
    import shutil
    import subprocess
    import tempfile

    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        path = os.path.join(td, "sample.bin")
        open(path, "wb").write(sample)
        cl = ",".join(str(c) for c in cpus)
        cmd = [sys.executable, os.path.abspath(__file__), "--cpu-child", path, str(level), cl, op, str(cap)]
        if shutil.which("taskset"):
            cmd = ["taskset", "-c", cl] + cmd
        r = subprocess.run(cmd, capture_output=True, text=True, check=True, timeout=600)
        res = json.loads(r.stdout.strip().splitlines()[-1])
        ref = open(path + ".ref", "rb").read() if os.path.exists(path + ".ref") else None
        return res["seconds"], ref


def cpu_and_parity(data, a, d_in):
    """Reference CPU timing on a bounded sample (pinned child processes), and GPU-vs-reference
    bytes on the 1-core sample."""
    from tests import oracles as O

    n = min(a.cpu_sample, len(data))
    sample = data[:n]
    allowed = sorted(os.sched_getaffinity(0))
    model = cpu_model()
    if O.has_ref():
        kind = "reference"
        cpu_s, ref_out = run_cpu_child(sample, a.level, allowed[:1])
    else:
        kind = "port"
        t = time.perf_counter()
        ref_out = O.orc_compress(sample, a.level)
        cpu_s = time.perf_counter() - t
    mt = None
    if O.has_ref() and a.cpu_threads > 1:
        cs = allowed[:a.cpu_threads]
        m = min(a.cpu_mt_sample, len(data))
        mt_s, _ = run_cpu_child(data[:m], a.level, cs)
        mt = {"value": round(m / mt_s / 1e6, 3), "unit": "MB/s", "cores": len(cs), "kind": "reference",
              "cpu_model": model, "pinned_cpus": f"{cs[0]}..{cs[-1]}" if len(cs) > 1 else str(cs[0]),
              "sample": f"first {m} B of the rank-0 input as {len(cs)} independent "
                        f"BZ2_bzBuffToBuffCompress -{a.level} streams on {len(cs)} pinned threads, {mt_s:.1f} s"}
    cap = B.bound(n)
    d_out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    nb, _, _ = B.compress_device(d_in.data_ptr(), n, a.level, d_out.data_ptr(), cap)
    torch.cuda.synchronize()
    gpu_sample = d_out[:nb].cpu().numpy().tobytes()
    return {
        "cpu_baseline": {"value": round(n / cpu_s / 1e6, 3), "unit": "MB/s", "cores": 1, "kind": kind,
                         "cpu_model": model, "pinned_cpus": str(allowed[0]),
                         "sample": f"first {n} B of the rank-0 input, BZ2_bzBuffToBuffCompress -{a.level}, "
                                   f"{cpu_s:.1f} s in a child process pinned to one core (taskset)"},
        "parity": {"sample_bytes": n, "bit_exact": gpu_sample == ref_out, "against": kind,
                   "out_bytes": len(ref_out)},
        **({"cpu_baseline_multicore": mt} if mt else {}),
    }


if __name__ == "__main__":
    if len(sys.argv) == 7 and sys.argv[1] == "--cpu-child":
        cpu_child(sys.argv[2], int(sys.argv[3]), sys.argv[4], sys.argv[5], int(sys.argv[6]))
    else:
        main()
