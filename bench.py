#!/usr/bin/env python3
"""Benchmark: pgnano C5 encode+decode throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): synthetic reads of 100,000 int16 samples (one POD5 chunk each,
below the 102,400 default chunk size), 100,000 reads per GPU, generated on the device by the same
integer-only generator the checker uses.  One step = encode every chunk + decode every blob, with
inputs already resident in HBM.  value = samples / (t_enc + t_dec) over all ranks (weak scaling:
each rank owns its own 100k-read shard; reads are assigned round-robin, read r -> rank r % N).

configs[3] (--global-reads 1000000): a fixed global read set split round-robin over the ranks
(strong scaling), each rank working through its share in resident batches of at most --reads reads.

Multi-GPU: one process per GPU.  Under torchrun the rank comes from the environment; `--gpus N`
without a torchrun environment starts N worker processes itself (before anything touches the GPU)
with the same environment torchrun would give them.  The only exchange is the final size/ratio
reduction (RCCL all-reduce over xGMI) and the max-over-ranks time.

The dominant kernel's roofline is measured live with HIP events on the launch stream; the CPU
baseline is the oracle (the libzstd-backed C restatement of the reference's C5 path) on one host
thread over a bounded sample, plus an all-cores leg (reads sharded over the box's CPU share).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--reads R] [--samples S] [--global-reads G]
"""
from __future__ import annotations

import argparse
import ctypes as C
import glob
import hashlib
import json
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MSamples/s encode+decode (1/2/4/8 GPU) at fixed ratio; % HBM roofline"
# synthetic-read dwell per pore chemistry (R9.4.1 ~9, R10.4.1 ~12.5 samples per level):
# p_switch in 1/65536 units
PORES = {"default": 6554, "r941": 7282, "r103": 6554, "r1041": 5243}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
# PMC traffic summaries (tools/traffic.sh) per workload, read into roofline.traffic when their
# source digest matches the kernels being run
TRAFFIC_FILES = {"configs[1]": "traffic_r06.json", "configs[4]": "traffic_r06_config4.json"}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--reads", type=int, default=None,
                   help="reads per GPU (default 100,000); with --global-reads: the largest batch a rank holds "
                        "(default: the rank's whole share when it fits --resident-gb of HBM)")
    p.add_argument("--resident-gb", type=float, default=200.0,
                   help="--global-reads: HBM a rank may hold for samples, blobs and decoded samples (6 B/sample)")
    p.add_argument("--samples", type=int, default=100_000, help="samples per read")
    p.add_argument("--global-reads", type=int, default=0,
                   help="configs[3]: a fixed global read count split round-robin over the ranks (strong scaling)")
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                   help="nccl (= RCCL) for one process per GPU; gloo lets several ranks share one GPU (rehearsal)")
    p.add_argument("--cpu-sample-reads", type=int, default=600)
    p.add_argument("--cpu-threads", type=int, default=0, help="all-cores CPU leg threads (0 = the box's CPU share)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-side", action="store_true",
                   help="skip the STREAM-copy, PCIe-inclusive and per-chunk side measurements (profiling runs: "
                        "the kernel statistics then hold only the bench batch's launches)")
    p.add_argument("--traffic-json", default=None,
                   help="PMC traffic summary (default: profiles/ file of this workload, TRAFFIC_FILES)")
    # the other BASELINE configs; the default run is configs[1]
    p.add_argument("--pore", choices=sorted(PORES), default="default",
                   help="generator parameters: dwell per pore chemistry (configs[2] uses r1041)")
    p.add_argument("--mixed-pores", action="store_true",
                   help="configs[4]: thirds of the reads with R9.4.1 / R10.3 / R10.4.1 parameters")
    p.add_argument("--decode-only", action="store_true", help="configs[4]: time the decode of the batch only")
    p.add_argument("--compare-vbz", action="store_true",
                   help="configs[2]: also encode the batch with VBZ (--VBZ) and report the size ratio")
    return p.parse_args(argv)


# ---- multi-process launch (no GPU in the parent) ------------------------------------------------
def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_workers(n: int, argv: list[str], script: str | None = None, timeout: float | None = None) -> int:
    """Start n worker processes of `script` (default: this file) with torchrun's environment (RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT) and wait for them.  The parent never
    touches the GPU; if a worker fails the others are terminated.  Returns the first non-zero exit
    status (0 when all succeed)."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", script or os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    t0 = time.monotonic()
    live = set(range(n))
    while live:
        for r in sorted(live):
            code = procs[r].poll()
            if code is None:
                continue
            live.discard(r)
            if code != 0 and rc == 0:
                rc = code
                for o in live:
                    procs[o].terminate()
        if timeout is not None and time.monotonic() - t0 > timeout and live:
            for o in live:
                procs[o].kill()
            rc = rc or 124
        time.sleep(0.05)
    return rc


# ---- read partition ---------------------------------------------------------------------------
def batch_cap(args) -> int:
    """Reads a rank holds at once: --reads, else (--global-reads) what fits --resident-gb of HBM
    (input samples, blobs at the plugin bound and decoded samples: 6 bytes per sample)."""
    if args.reads is not None:
        return args.reads
    if args.global_reads <= 0:
        return 100_000
    return max(1, int(args.resident_gb * 1e9 // (6 * max(args.samples, 1))))


def rank_batches(args, rank: int, world: int):
    """(reads of this rank, [reads per batch], scaling).  Weak scaling (default): every rank owns
    --reads reads.  Strong scaling (--global-reads G): rank r owns the global reads r, r + N, ...
    below G: all of them resident when they fit (batch_cap), else in equal batches of distinct reads
    (batch b holds the rank's reads b * B .. (b + 1) * B - 1, generated before it is timed)."""
    cap = batch_cap(args)
    if args.global_reads <= 0:
        return cap, [cap], "weak"
    mine = max(0, (args.global_reads - rank + world - 1) // world)
    if mine == 0:
        return 0, [], "strong"
    nb = (mine + cap - 1) // cap
    base, extra = divmod(mine, nb)
    return mine, [base + (1 if i < extra else 0) for i in range(nb)], "strong"


# ---- CPU baselines (the oracle, a C restatement of C5.hpp over libzstd: test infrastructure, timed as the CPU baseline) ---
def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O

    return O


def cpu_baseline(samples_per_read: int, nreads: int, seed: int):
    """Oracle (C restatement of C5.hpp:282-683 over libzstd 1.4.x) on one host thread."""
    import numpy as np

    O = _oracle()
    L = O.oracle()
    xs = [O.synth_read(r, samples_per_read, seed=seed) for r in range(nreads)]
    cap = L.pgno_c5_bound(samples_per_read)
    out = np.zeros(cap, np.uint8)
    back = np.zeros(samples_per_read, np.int16)
    ol = C.c_size_t(0)
    blobs = []
    t0 = time.perf_counter()
    for x in xs:
        rc = L.pgno_c5_compress(x.ctypes.data, x.size, out.ctypes.data, cap, C.byref(ol), None)
        assert rc == 0
        blobs.append(out[: ol.value].copy())
    t1 = time.perf_counter()
    for b in blobs:
        rc = L.pgno_c5_decompress(b.ctypes.data, b.size, back.ctypes.data, samples_per_read)
        assert rc == 0
    t2 = time.perf_counter()
    n = samples_per_read * nreads
    return {
        "value": n / ((t1 - t0) + (t2 - t1)) / 1e6,
        "unit": "MSamples/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{nreads} synthetic reads x {samples_per_read} samples (same generator), oracle C5 "
                  f"encode {n / (t1 - t0) / 1e6:.1f} + decode {n / (t2 - t1) / 1e6:.1f} MS/s, "
                  f"libzstd {L.pgno_zstd_version()}",
    }


def cpu_share() -> int:
    """Host threads this process may use: the box's CPU share (OMP_NUM_THREADS is set to it on the
    GPU boxes), else the affinity mask."""
    v = os.environ.get("OMP_NUM_THREADS")
    if v and v.isdigit() and int(v) > 0:
        return int(v)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline_all_cores(samples_per_read: int, reads_per_thread: int, seed: int, threads: int):
    """The same oracle path on `threads` host threads, reads sharded round-robin (ctypes releases the
    GIL inside the C calls).  Encode and decode phases are timed separately, each from a barrier."""
    import numpy as np

    O = _oracle()
    L = O.oracle()
    cap = L.pgno_c5_bound(samples_per_read)
    xs = [None] * threads
    blobs = [[None] * reads_per_thread for _ in range(threads)]
    bar = threading.Barrier(threads + 1)
    errors = []

    def work(t):
        try:
            # this thread's reads t, t + threads, ... (generated here, outside the timed phases)
            xs[t] = [O.synth_read(t + threads * k, samples_per_read, seed=seed) for k in range(reads_per_thread)]
            out = np.zeros(cap, np.uint8)
            back = np.zeros(samples_per_read, np.int16)
            ol = C.c_size_t(0)
            bar.wait()
            for k, x in enumerate(xs[t]):
                if L.pgno_c5_compress(x.ctypes.data, x.size, out.ctypes.data, cap, C.byref(ol), None) != 0:
                    errors.append("encode")
                blobs[t][k] = out[: ol.value].copy()
            bar.wait()
            bar.wait()
            for b in blobs[t]:
                if L.pgno_c5_decompress(b.ctypes.data, b.size, back.ctypes.data, samples_per_read) != 0:
                    errors.append("decode")
            bar.wait()
        except threading.BrokenBarrierError:
            errors.append("barrier")

    ths = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for th in ths:
        th.start()
    bar.wait()
    t0 = time.perf_counter()
    bar.wait()
    t1 = time.perf_counter()
    bar.wait()
    t2 = time.perf_counter()
    bar.wait()
    t3 = time.perf_counter()
    for th in ths:
        th.join()
    assert not errors, errors
    n = samples_per_read * reads_per_thread * threads
    te, td = t1 - t0, t3 - t2
    return {
        "value": n / (te + td) / 1e6,
        "unit": "MSamples/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{threads} threads x {reads_per_thread} synthetic reads x {samples_per_read} samples, oracle C5 "
                  f"encode {n / te / 1e6:.1f} + decode {n / td / 1e6:.1f} MS/s",
    }


def host_info():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model, os.cpu_count()


# ---- side measurements (rank 0, N = 1) --------------------------------------------------------
def stream_copy_gbs(torch, nbytes=4 << 30, reps=5):
    """Device STREAM-copy ceiling: read + write bytes of a large device-to-device copy."""
    a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    del a, b
    return 2.0 * nbytes / (ms * 1e-3) / 1e9


def pcie_inclusive(torch, codec, S, seed, nreads=2000):
    """Host-memory rates (pinned buffers, not part of `value`): H2D samples + encode + D2H blobs,
    and H2D blobs + decode + D2H samples, on a sample of the same workload."""
    samples, offs, counts = codec.synth_reads(nreads, S, seed=seed)
    enc = codec.compress_batch(samples, offs, counts)
    torch.cuda.synchronize()
    h_samples = samples.cpu().pin_memory()
    h_blobs = enc.blobs.cpu().pin_memory()
    h_back = torch.empty_like(h_samples).pin_memory()
    d_samples = torch.empty_like(samples)
    d_blobs = torch.empty_like(enc.blobs)
    out = torch.empty_like(samples)
    n = nreads * S
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d_samples.copy_(h_samples, non_blocking=True)
    e2 = codec.compress_batch(d_samples, offs, counts, out=d_blobs, out_offsets=enc.offsets, out_caps=enc.caps)
    h_blobs.copy_(d_blobs, non_blocking=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    d_blobs.copy_(h_blobs, non_blocking=True)
    codec.decompress_batch(d_blobs, enc.offsets, e2.sizes, counts, out=out, out_offsets=offs)
    h_back.copy_(out, non_blocking=True)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return {"encode_msamples_s": round(n / (t1 - t0) / 1e6, 1), "decode_msamples_s": round(n / (t2 - t1) / 1e6, 1),
            "sample": f"{nreads} reads x {S} samples, pinned host buffers"}


def per_chunk_plugin(torch, codec, S, seed, nreads=200):
    """The drop-in per-chunk surface as the reference's writer/reader call it (one chunk per call,
    host memory, synchronous: pgn_compress_signal / pgn_decompress_signal)."""
    samples, offs, counts = codec.synth_reads(nreads, S, seed=seed)
    host = samples.cpu().numpy()
    torch.cuda.synchronize()
    xs = [host[r * S:(r + 1) * S] for r in range(nreads)]
    codec.decompress_signal(codec.compress_signal(xs[0]), sample_count=S)  # warm the staging buffers
    t0 = time.perf_counter()
    blobs = [codec.compress_signal(x) for x in xs]
    t1 = time.perf_counter()
    for b in blobs:
        codec.decompress_signal(b, sample_count=S)
    t2 = time.perf_counter()
    n = nreads * S
    return {"encode_msamples_s": round(n / (t1 - t0) / 1e6, 1), "decode_msamples_s": round(n / (t2 - t1) / 1e6, 1),
            "calls_per_s": round(nreads / (t1 - t0), 1),
            "sample": f"{nreads} reads x {S} samples, one pgn_compress_signal / pgn_decompress_signal call each"}


def per_chunk_plugin_threads(torch, codec, S, seed, nthreads=16, nreads=1600):
    """The per-chunk surface under concurrent callers on one context (the reference's reader calls
    it from the async signal loader's worker threads, async_signal_loader.cpp:174-208): nthreads
    host threads, each one chunk per call; calls that meet on the device are combined into one
    small batch (pgn_kernels.hip PcArena)."""
    import threading

    samples, offs, counts = codec.synth_reads(nreads, S, seed=seed)
    host = samples.cpu().numpy()
    torch.cuda.synchronize()
    xs = [host[r * S:(r + 1) * S] for r in range(nreads)]
    blobs = [None] * nreads
    ok = [True]

    def run(fn):
        def work(i):
            for r in range(i, nreads, nthreads):
                fn(r)
        ts = [threading.Thread(target=work, args=(i,)) for i in range(nthreads)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        return time.perf_counter() - t0

    def enc(r):
        blobs[r] = codec.compress_signal(xs[r])

    def dec(r):
        y = codec.decompress_signal(blobs[r], sample_count=S)
        if r % 97 == 0 and not (y == xs[r]).all():
            ok[0] = False

    run(lambda r: enc(r) if r < 2 * nthreads else None)  # warm the arenas
    te = run(enc)
    td = run(dec)
    n = nreads * S
    return {"encode_msamples_s": round(n / te / 1e6, 1), "decode_msamples_s": round(n / td / 1e6, 1),
            "threads": nthreads, "round_trip_ok": ok[0],
            "sample": f"{nreads} reads x {S} samples over {nthreads} host threads on one context, "
                      "one pgn_compress_signal / pgn_decompress_signal call each"}


def pod5_batch_host(torch, codec, S, seed, nreads=1000):
    """The batched POD5 integration (include/pgnano_pod5.h) on host memory: one
    pod5_add_reads_data-shaped call (reads chunked at the writer's 102,400 samples, all chunks in one
    launch, the packed signal column back) and the decode of those rows, PCIe transfers included."""
    import numpy as np

    from rawnanoporesignalcompression_amd import Pod5SignalBatch

    samples, _, _ = codec.synth_reads(nreads, S, seed=seed)
    host = samples.cpu().numpy()
    torch.cuda.synchronize()
    reads = [host[r * S:(r + 1) * S] for r in range(nreads)]
    out = np.zeros(nreads * S, dtype=np.int16)  # the reader's destination (touched: no first-touch faults)
    b = Pod5SignalBatch(codec)
    te, td = [], []
    try:
        offsets, data, smp, _ = b.compress_reads(reads, copy=False)  # staging buffers at full size
        b.decompress_rows(offsets.copy(), data.copy(), smp.copy(), out=out)
        for _ in range(3):
            t0 = time.perf_counter()
            offsets, data, smp, _ = b.compress_reads(reads, copy=False)
            te.append(time.perf_counter() - t0)
            offsets, data, smp = offsets.copy(), data.copy(), smp.copy()  # the writer's column, untimed
            t0 = time.perf_counter()
            b.decompress_rows(offsets, data, smp, out=out)
            td.append(time.perf_counter() - t0)
        ok = bool(np.array_equal(out, host[: nreads * S]))
    finally:
        b.close()
    n = nreads * S
    return {"encode_msamples_s": round(n / min(te) / 1e6, 1), "decode_msamples_s": round(n / min(td) / 1e6, 1),
            "round_trip_ok": ok,
            "sample": f"{nreads} reads x {S} samples per pgn_pod5_compress_reads / pgn_pod5_decompress_rows call "
                      "(best of 3 after a full-size warm-up), host memory: pageable reads in, the column's packed "
                      "bytes back, samples into the caller's buffer; pinned staging inside"}


# ---- roofline traffic evidence -------------------------------------------------------------------
def source_digest() -> str:
    """sha256 over the kernel sources the measured library is built from (csrc/*.hip, csrc/*.h,
    include/*.h): a traffic file measured on other sources is stale."""
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "rawnanoporesignalcompression_amd", "csrc", "*.hip")) +
                   glob.glob(os.path.join(ROOT, "rawnanoporesignalcompression_amd", "csrc", "*.h")) +
                   glob.glob(os.path.join(ROOT, "include", "*.h")))
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def load_traffic(path, R, S, dominant, workload):
    """(bytes per launch of the dominant direction, provenance) from the committed PMC summary, or
    (None, reason) when it does not apply to this run (workload: "configs[1]" / "configs[4]", None =
    no measured file applies) or was measured on other kernel sources."""
    try:
        with open(path) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        return None, f"no traffic file {os.path.relpath(path, ROOT)}"
    if (workload is None or tj.get("workload", "configs[1]") != workload or tj.get("reads") != R
            or tj.get("samples") != S):
        return None, "traffic file measured on another workload"
    if tj.get("source_sha256") != source_digest():
        return None, "stale: traffic file measured on other kernel sources"
    return tj.get(dominant), os.path.relpath(path, ROOT)


# ---- one rank ---------------------------------------------------------------------------------
def run_rank(args, rank, world, local, codec, torch, dist, device="cuda", cuda=True):
    """The timed body of one rank: generate this rank's reads (resident), warm up, time exactly
    --steps steps between barriers + device synchronisation, reduce counters (SUM) and time (MAX)
    over the ranks.  Returns the bench line on rank 0, else None.  `codec` is the device codec
    (PGNanoCodec); the CPU tests pass a stand-in with the same methods."""
    from rawnanoporesignalcompression_amd.shard import reduce_run, shard_reads

    sync = torch.cuda.synchronize if cuda else (lambda: None)
    S = args.samples
    mine, batches, scaling = rank_batches(args, rank, world)
    B = max(batches) if batches else 0
    starts = [sum(batches[:b]) for b in range(len(batches))]  # the rank's read index of each batch's first read
    sh = shard_reads(B, rank, world)
    samples = torch.empty(max(B * S, 1), dtype=torch.int16, device=device)
    counts = torch.full((B,), S, dtype=torch.int32, device=device)
    offs = torch.arange(B, dtype=torch.int64, device=device) * S

    def generate(b):
        """batch b's reads: this rank's reads starts[b] .. (global ids first_read + k * stride)"""
        nb, first = batches[b], sh.first_read + starts[b] * sh.read_stride
        if args.mixed_pores:  # thirds of the batch per chemistry
            cuts = [0, nb // 3, 2 * nb // 3, nb]
            for i, pore in enumerate(("r941", "r103", "r1041")):
                a, e = cuts[i], cuts[i + 1]
                codec.synth_reads(e - a, S, seed=args.seed, first_read=first + a * sh.read_stride,
                                  read_stride=sh.read_stride, p_switch_q16=PORES[pore], out=samples[a * S:e * S])
        else:
            codec.synth_reads(nb, S, seed=args.seed, first_read=first, read_stride=sh.read_stride,
                              p_switch_q16=PORES[args.pore], out=samples[: nb * S])

    if B:
        generate(0)
    sync()
    caps = torch.clamp(counts.to(torch.int64) * 2 + 26, min=1024)
    boffs = torch.zeros(B, dtype=torch.int64, device=device)
    if B > 1:
        boffs[1:] = torch.cumsum(caps, 0)[:-1]
    blobs = torch.empty(max(int(caps.sum().item()), 1), dtype=torch.uint8, device=device)
    decoded = torch.empty(max(B * S, 1), dtype=torch.int16, device=device)
    enc_ms, dec_ms = [], []
    state = {"ok": True, "bytes": [0] * len(batches)}

    def encode(nb):
        return codec.compress_batch(samples[: nb * S], offs[:nb], counts[:nb], out=blobs, out_offsets=boffs[:nb],
                                    out_caps=caps[:nb], stream=codec.stream)

    def decode(nb, sizes):
        codec.decompress_batch(blobs, boffs[:nb], sizes, counts[:nb], out=decoded, out_offsets=offs[:nb],
                               stream=codec.stream)

    def barrier():
        sync()
        if world > 1:
            dist.barrier()
        sync()

    if args.decode_only and B:  # configs[4]: the blobs are made once, outside the timed region
        state["enc0"] = encode(B)
        sync()

    # One step = every batch of the rank encoded and decoded.  A single batch stays resident: the step
    # is exactly the timed region.  Several batches (a share too large for HBM): each batch's reads are
    # generated outside the timing, and the step's time is the sum of its batches' timed sections, each
    # bracketed by a barrier and device synchronisation.
    def step(timed):
        e = d = t = 0.0
        for b, nb in enumerate(batches):
            if len(batches) > 1:
                generate(b)
                if args.decode_only:  # this batch's blobs, untimed
                    state["enc0"] = encode(nb)
            barrier()
            t0 = time.perf_counter()
            if args.decode_only:
                enc = state["enc0"]
                decode(nb, enc.sizes[:nb])
                d += codec.last_decode_ms()
            else:
                enc = encode(nb)
                decode(nb, enc.sizes)
                e += codec.last_encode_ms()
                d += codec.last_decode_ms()
            barrier()
            t += time.perf_counter() - t0
            if timed:  # correctness and the measured compressed bytes of every batch (untimed)
                state["ok"] &= bool((enc.status[:nb] == 0).all().item()) and bool(
                    torch.equal(decoded[: nb * S], samples[: nb * S]))
                state["bytes"][b] = int(enc.sizes[:nb].sum().item())
        if timed:
            enc_ms.append(e)
            dec_ms.append(d)
        return t

    for _ in range(args.warmup):
        step(False)
    elapsed = sum(step(True) for _ in range(args.steps))
    ok = state["ok"]
    comp_rank = sum(state["bytes"])
    red_dev = device if (cuda and args.dist_backend == "nccl") else "cpu"
    tot, elapsed = reduce_run({"compressed_bytes": comp_rank, "samples": mine * S, "errors": 0 if ok else 1,
                               "chunks": mine}, elapsed, device=red_dev)
    if rank != 0:
        return None
    comp_total, samples_total, errors = tot["compressed_bytes"], tot["samples"], tot["errors"]
    ms_per_step = 1e3 * elapsed / args.steps
    value = samples_total * args.steps / elapsed / 1e6
    c_per_sample = comp_total / max(samples_total, 1)
    e_ms = sum(enc_ms) / len(enc_ms)
    d_ms = sum(dec_ms) / len(dec_ms)
    # the roofline is taken over the dominant direction's launch sequence (HIP events on the codec
    # stream around all its kernels) of this rank's first batch
    R0 = batches[0] if batches else 0
    dominant = "c5_decode" if (d_ms >= e_ms or args.decode_only) else "c5_encode"
    kernels = codec.kernels(1 if dominant == "c5_decode" else 0)
    k_ms = (d_ms if args.decode_only else max(e_ms, d_ms)) / max(len(batches), 1) if batches else 0.0
    algo_bytes = (2.0 + c_per_sample) * R0 * S  # per launch (encode 2 + C, decode C + 2 per sample)
    achieved = algo_bytes / (k_ms * 1e-3) / 1e9 if k_ms > 0 else 0.0
    if args.mixed_pores and args.decode_only:
        wl = "configs[4]"
    elif not (args.mixed_pores or args.pore != "default" or args.decode_only):
        wl = "configs[1]"
    else:
        wl = None
    tpath = args.traffic_json or os.path.join(ROOT, "profiles", TRAFFIC_FILES.get(wl, TRAFFIC_FILES["configs[1]"]))
    traffic, traffic_src = load_traffic(tpath, R0, S, dominant, wl)
    if args.mixed_pores:
        gen = "configs[4]: mixed pores (thirds R9.4.1 / R10.3 / R10.4.1 generator dwell)"
    elif args.pore != "default":
        gen = f"configs[2]: {args.pore} generator dwell"
    elif args.global_reads > 0:
        gen = f"configs[3]: {args.global_reads} global reads round-robin over {world} GPU(s)"
    else:
        gen = "configs[1]"
    what = "C5 decode only" if args.decode_only else "C5 encode+decode"
    if args.global_reads > 0:
        shape = (f"{gen}: {args.global_reads} reads x {S} int16 samples in total (1 chunk each), "
                 + ("the rank's share resident" if len(batches) <= 1 else f"batches of <= {B} distinct reads per GPU")
                 + f", {what}")
    else:
        shape = f"{gen}: {B} reads x {S} int16 samples per GPU (1 chunk each), {what}"
    data = "synthetic (device generator: piecewise-constant levels + N(0,12) noise, integer-only)"
    if len(batches) > 1:
        data += (f"; {len(batches)} batches of distinct reads per rank, each generated outside the timing "
                 "(the step time is the sum of the batches' timed sections)")
    return {
        "metric": METRIC if not args.decode_only else "MSamples/s decode (configs[4]); % HBM roofline",
        "value": round(value, 2),
        "unit": "MSamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "int16",
        "data": data,
        "config": {
            "workload": shape,
            "reads_per_gpu": mine,
            "samples_per_read": S,
            "global_reads": samples_total // max(S, 1),
            "parallelism": f"dp{world} (reads round-robin, no data-path collective)",
        },
        "encode_ms": round(e_ms, 3),
        "decode_ms": round(d_ms, 3),
        "encode_msamples_s": round(mine * S / e_ms / 1e3, 1) if e_ms > 0 else None,
        "decode_msamples_s": round(mine * S / d_ms / 1e3, 1) if d_ms > 0 else None,
        "bits_per_sample": round(8.0 * c_per_sample, 4),
        "compressed_bytes": comp_total,
        "round_trip_ok": errors == 0,
        "roofline": {
            "bound": "hbm",
            "kernel": dominant,
            "kernels": kernels,
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
        },
    }


def main(argv=None):
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `bench.py --gpus N` outside torchrun: start the N ranks here, before anything touches the GPU
        sys.exit(launch_workers(args.gpus, sys.argv[1:] if argv is None else list(argv)))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus not in (1, world):
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    ndev = torch.cuda.device_count()
    dev_index = local % max(ndev, 1)  # gloo rehearsals may put several ranks on one GPU
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group("gloo")
    torch.cuda.set_device(dev_index)
    from rawnanoporesignalcompression_amd import PGNanoCodec

    codec = PGNanoCodec(dev_index)
    side = {}
    if rank == 0 and world == 1 and not args.no_side:
        side["stream_copy_gbs"] = round(stream_copy_gbs(torch), 1)
        side["pcie_inclusive"] = pcie_inclusive(torch, codec, args.samples, args.seed)
        side["per_chunk_plugin"] = per_chunk_plugin(torch, codec, args.samples, args.seed)
        side["per_chunk_plugin_threads"] = per_chunk_plugin_threads(torch, codec, args.samples, args.seed)
        side["pod5_batch_host"] = pod5_batch_host(torch, codec, args.samples, args.seed)
    line = run_rank(args, rank, world, local, codec, torch, dist, device=torch.device("cuda", dev_index))
    if line is not None:
        line.update(side)
        R, S = batch_cap(args), args.samples
        if args.compare_vbz and world == 1:  # the --VBZ side of the ratio comparison, outside the timing
            from rawnanoporesignalcompression_amd import VBZCodec

            samples = torch.empty(R * S, dtype=torch.int16, device="cuda")
            _, offs, counts = codec.synth_reads(R, S, seed=args.seed, p_switch_q16=PORES[args.pore], out=samples)
            vz = VBZCodec(dev_index)
            ev = vz.compress_batch(samples, offs, counts)
            torch.cuda.synchronize()
            vbytes = int(ev.sizes.sum().item())
            c5bytes = line["compressed_bytes"]
            line["vbz"] = {"bits_per_sample": round(8.0 * vbytes / (R * S), 4),
                           "c5_vs_vbz_ratio": round(c5bytes / max(vbytes, 1), 4),
                           "status_ok": bool((ev.status == 0).all().item())}
            vz.close()
            del samples
        if not args.no_cpu_baseline and world == 1:
            model, ncpu = host_info()
            line["cpu_baseline"] = cpu_baseline(S, args.cpu_sample_reads, args.seed)
            line["cpu_baseline"]["sample"] += f"; host {model}, {ncpu} logical CPUs"
            threads = args.cpu_threads or cpu_share()
            line["cpu_baseline_all_cores"] = cpu_baseline_all_cores(S, max(8, 4 * args.cpu_sample_reads // threads),
                                                                    args.seed, threads)
            line["cpu_baseline_all_cores"]["sample"] += f"; host {model}, {ncpu} logical CPUs, CPU share {threads}"
        elif not args.no_cpu_baseline:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    codec.close()


if __name__ == "__main__":
    main()
