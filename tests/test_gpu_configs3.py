"""configs[3] on the HIP codec (BASELINE.json: 1M reads round-robin over the GPUs, strong scaling).

`bench.run_rank` with --global-reads drives the real PGNanoCodec on two gloo ranks that share cuda:0:
each rank owns the global reads r, r + 2, ... and, with --reads below its share, walks them in
several batches of distinct reads (the sharding unit of the reference's writer is the read batch,
pod5/c++/pod5_format/c_api.cpp:1104-1129).  Checked against the oracle: the round trip, the total
compressed bytes over all G reads, and sampled blobs of every batch, whose inputs must be the
generator's reads of the rank's global ids.  The 8-GPU scaling curve itself is the driver's run.
"""
import os
import socket
import sys

import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu

G, R, S = 2001, 600, 100_000


class _Recorder:
    """The codec with compress_batch checked on a sample of each batch (outside bench's concerns:
    the check runs after the call, on host copies)."""

    def __init__(self, codec, rank, world):
        self._c, self.rank, self.world = codec, rank, world
        self.done = 0           # reads of this rank encoded so far (batches come in order)
        self.checked = []       # (global id, blob equal, input equal)
        self.first_step = True

    def __getattr__(self, k):
        return getattr(self._c, k)

    def compress_batch(self, samples, offs, counts, **kw):
        import torch

        enc = self._c.compress_batch(samples, offs, counts, **kw)
        if not self.first_step:
            return enc
        torch.cuda.synchronize()
        nb = int(counts.numel())
        out, oo = kw["out"], kw["out_offsets"]
        for j in sorted({0, nb // 2, nb - 1}):
            gid = self.rank + self.world * (self.done + j)
            x = samples[j * S:(j + 1) * S].cpu().numpy()
            lo, n = int(oo[j].item()), int(enc.sizes[j].item())
            blob = out[lo:lo + n].cpu().numpy().tobytes()
            rc, ref, _ = O.c5_compress(x)
            self.checked.append((gid, rc == 0 and blob == ref, bool(np.array_equal(x, O.synth_read(gid, S)))))
        self.done += nb
        if self.done >= (G - self.rank + self.world - 1) // self.world:
            self.first_step = False
        return enc


def _rank(rank, world, port, q):
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    import torch
    import torch.distributed as dist

    import bench
    from rawnanoporesignalcompression_amd import PGNanoCodec

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    codec = None
    try:
        torch.cuda.set_device(0)
        codec = PGNanoCodec(0)
        rec = _Recorder(codec, rank, world)
        args = bench.parse(["--global-reads", str(G), "--reads", str(R), "--samples", str(S), "--steps", "1",
                            "--warmup", "0", "--dist-backend", "gloo", "--no-side", "--no-cpu-baseline"])
        line = bench.run_rank(args, rank, world, 0, rec, torch, dist, device=torch.device("cuda", 0))
        q.put((rank, "ok", line, rec.checked, bench.rank_batches(args, rank, world)[1]))
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        q.put((rank, "error", f"{type(e).__name__}: {e}", None, None))
    finally:
        if codec is not None:
            codec.close()
        dist.destroy_process_group()


def test_configs3_global_reads_two_ranks_on_hip_codec():
    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=110) for _ in range(2)), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert all(r[1] == "ok" for r in res), res
    line = res[0][2]
    # every rank walked its share in several batches of distinct reads
    assert res[0][4] == [501, 500] and res[1][4] == [500, 500]
    assert line["scaling"] == "strong" and line["n_gpus"] == 2
    assert line["config"]["global_reads"] == G and line["round_trip_ok"]
    # the sampled blobs equal the oracle's, on the generator's reads of the rank's global ids
    for _, _, _, checked, _ in res:
        assert len(checked) == 6 and all(b and x for _, b, x in checked), checked
    # the job's compressed bytes are the oracle's over all G reads
    ref = sum(len(O.c5_compress(O.synth_read(i, S))[1]) for i in range(G))
    assert line["compressed_bytes"] == ref
