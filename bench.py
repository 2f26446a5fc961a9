#!/usr/bin/env python3
"""Benchmark: pgnano C5 encode+decode throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): synthetic reads of 100,000 int16 samples (one POD5 chunk each,
below the 102,400 default chunk size), 100,000 reads per GPU, generated on the device by the same
integer-only generator the checker uses.  One step = encode every chunk + decode every blob, with
inputs already resident in HBM.  value = samples / (t_enc + t_dec) over all ranks (weak scaling:
each rank owns its own 100k-read shard; reads are assigned round-robin, read r -> rank r % N).

The dominant kernel's roofline is measured live with HIP events on the launch stream; the CPU
baseline is the oracle (the libzstd-backed C restatement of the reference's C5 path) on one host
thread over a bounded sample.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--reads R] [--samples S]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MSamples/s encode+decode (1/2/4/8 GPU) at fixed ratio; % HBM roofline"
# synthetic-read dwell per pore chemistry (R9.4.1 ~9, R10.4.1 ~12.5 samples per level):
# p_switch in 1/65536 units
PORES = {"default": 6554, "r941": 7282, "r103": 6554, "r1041": 5243}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--reads", type=int, default=100_000, help="reads per GPU")
    p.add_argument("--samples", type=int, default=100_000, help="samples per read")
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--cpu-sample-reads", type=int, default=600)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-side", action="store_true",
                   help="skip the STREAM-copy and PCIe-inclusive side measurements (profiling runs: the "
                        "kernel statistics then hold only the bench batch's launches)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r01.json"))
    # the other BASELINE configs; the default run is configs[1]
    p.add_argument("--pore", choices=sorted(PORES), default="default",
                   help="generator parameters: dwell per pore chemistry (configs[2] uses r1041)")
    p.add_argument("--mixed-pores", action="store_true",
                   help="configs[4]: thirds of the reads with R9.4.1 / R10.3 / R10.4.1 parameters")
    p.add_argument("--decode-only", action="store_true", help="configs[4]: time the decode of the batch only")
    p.add_argument("--compare-vbz", action="store_true",
                   help="configs[2]: also encode the batch with VBZ (--VBZ) and report the size ratio")
    return p.parse_args()


def cpu_baseline(samples_per_read: int, nreads: int, seed: int):
    """Oracle (C restatement of C5.hpp:282-683 over libzstd 1.4.x) on one host thread."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import _oracle as O

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


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    from rawnanoporesignalcompression_amd import PGNanoCodec
    from rawnanoporesignalcompression_amd.shard import reduce_run, shard_reads

    codec = PGNanoCodec(local)
    R, S = args.reads, args.samples
    side = {}
    if rank == 0 and world == 1 and not args.no_side:
        side["stream_copy_gbs"] = round(stream_copy_gbs(torch), 1)
        side["pcie_inclusive"] = pcie_inclusive(torch, codec, S, args.seed)
    # this rank's shard: global reads rank, rank + world, ... (round-robin)
    sh = shard_reads(R, rank, world)
    samples = torch.empty(R * S, dtype=torch.int16, device="cuda")
    counts = torch.full((R,), S, dtype=torch.int32, device="cuda")
    offs = torch.arange(R, dtype=torch.int64, device="cuda") * S
    if args.mixed_pores:  # thirds of the shard per chemistry
        cuts = [0, R // 3, 2 * R // 3, R]
        for i, pore in enumerate(("r941", "r103", "r1041")):
            a, b = cuts[i], cuts[i + 1]
            codec.synth_reads(b - a, S, seed=args.seed, first_read=sh.first_read + a * sh.read_stride,
                              read_stride=sh.read_stride, p_switch_q16=PORES[pore], out=samples[a * S:b * S])
    else:
        codec.synth_reads(R, S, seed=args.seed, first_read=sh.first_read, read_stride=sh.read_stride,
                          p_switch_q16=PORES[args.pore], out=samples)
    torch.cuda.synchronize()
    caps = torch.clamp(counts.to(torch.int64) * 2 + 26, min=1024)
    boffs = torch.zeros(R, dtype=torch.int64, device="cuda")
    boffs[1:] = torch.cumsum(caps, 0)[:-1]
    blobs = torch.empty(int(caps.sum().item()), dtype=torch.uint8, device="cuda")
    decoded = torch.empty(R * S, dtype=torch.int16, device="cuda")

    def step():
        enc = codec.compress_batch(samples, offs, counts, out=blobs, out_offsets=boffs, out_caps=caps,
                                   stream=codec.stream)
        codec.decompress_batch(blobs, boffs, enc.sizes, counts, out=decoded, out_offsets=offs,
                               stream=codec.stream)
        return enc

    if args.decode_only:  # configs[4]: the blobs are made once, outside the timed region
        enc0 = codec.compress_batch(samples, offs, counts, out=blobs, out_offsets=boffs, out_caps=caps,
                                    stream=codec.stream)
        torch.cuda.synchronize()

        def step():  # noqa: F811
            codec.decompress_batch(blobs, boffs, enc0.sizes, counts, out=decoded, out_offsets=offs,
                                   stream=codec.stream)
            return enc0

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    enc_ms, dec_ms = [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        enc = step()
        enc_ms.append(codec.last_encode_ms())
        dec_ms.append(codec.last_decode_ms())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # correctness of the timed work (outside the timed region)
    ok = bool((enc.status == 0).all().item()) and bool(torch.equal(decoded, samples))
    comp_bytes = int(enc.sizes.sum().item())
    # the final size/ratio reduction (RCCL over xGMI) and the max-over-ranks time
    tot, elapsed = reduce_run({"compressed_bytes": comp_bytes, "samples": R * S, "errors": 0 if ok else 1,
                               "chunks": R}, elapsed, device="cuda")
    comp_total, samples_total, errors = tot["compressed_bytes"], tot["samples"], tot["errors"]
    if rank == 0:
        ms_per_step = 1e3 * elapsed / args.steps
        value = samples_total * args.steps / elapsed / 1e6
        c_per_sample = comp_total / samples_total
        e_ms = sum(enc_ms) / len(enc_ms)
        d_ms = sum(dec_ms) / len(dec_ms)
        # the hot path is a three-kernel pipeline per direction; the roofline is taken over the dominant
        # direction's launch sequence (HIP events on the codec stream around all its kernels)
        dominant = "c5_decode" if (d_ms >= e_ms or args.decode_only) else "c5_encode"
        kernels = codec.kernels(1 if dominant == "c5_decode" else 0)
        k_ms = d_ms if args.decode_only else max(e_ms, d_ms)
        algo_bytes = (2.0 + comp_bytes / (R * S)) * R * S  # per launch on this GPU
        achieved = algo_bytes / (k_ms * 1e-3) / 1e9
        traffic = None
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("reads") == R and tj.get("samples") == S and not (args.mixed_pores or args.pore != "default"):
                traffic = tj.get(dominant)
        except (OSError, ValueError):
            pass
        if args.mixed_pores:
            gen = "configs[4]: mixed pores (thirds R9.4.1 / R10.3 / R10.4.1 generator dwell)"
        elif args.pore != "default":
            gen = f"configs[2]: {args.pore} generator dwell"
        else:
            gen = "configs[1]"
        what = "C5 decode only" if args.decode_only else "C5 encode+decode"
        line = {
            "metric": METRIC if not args.decode_only else "MSamples/s decode (configs[4]); % HBM roofline",
            "value": round(value, 2),
            "unit": "MSamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int16",
            "data": "synthetic (device generator: piecewise-constant levels + N(0,12) noise, integer-only)",
            "config": {
                "workload": f"{gen}: {R} reads x {S} int16 samples per GPU (1 chunk each), {what}",
                "reads_per_gpu": R,
                "samples_per_read": S,
                "parallelism": f"dp{world} (reads round-robin, no data-path collective)",
            },
            "encode_ms": round(e_ms, 3),
            "decode_ms": round(d_ms, 3),
            "encode_msamples_s": round(R * S / e_ms / 1e3, 1),
            "decode_msamples_s": round(R * S / d_ms / 1e3, 1),
            "bits_per_sample": round(8.0 * c_per_sample, 4),
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
            },
        }
        line.update(side)
        if args.compare_vbz and world == 1:  # the --VBZ side of the ratio comparison, outside the timing
            from rawnanoporesignalcompression_amd import VBZCodec

            vz = VBZCodec(local)
            ev = vz.compress_batch(samples, offs, counts)
            torch.cuda.synchronize()
            vbytes = int(ev.sizes.sum().item())
            line["vbz"] = {"bits_per_sample": round(8.0 * vbytes / (R * S), 4),
                           "c5_vs_vbz_ratio": round(comp_bytes / max(vbytes, 1), 4),
                           "status_ok": bool((ev.status == 0).all().item())}
            vz.close()
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(S, args.cpu_sample_reads, args.seed) if world == 1 else None
            if line["cpu_baseline"]:
                model, ncpu = host_info()
                line["cpu_baseline"]["sample"] += f"; host {model}, {ncpu} logical CPUs"
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    codec.close()


if __name__ == "__main__":
    main()
