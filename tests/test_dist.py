"""N > 1 path on CPU: two gloo ranks shard reads round-robin, encode their shard (oracle on CPU,
standing in for the device codec), and reduce sizes exactly as bench.py does."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, reads, n, q):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    import torch.distributed as dist

    import _oracle as O
    from rawnanoporesignalcompression_amd.shard import reduce_run, shard_reads

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = shard_reads(reads, rank, world)
    comp = 0
    for gid in sh.global_ids():
        rc, blob, _ = O.c5_compress(O.synth_read(gid, n))
        assert rc == 0
        comp += len(blob)
    tot, t = reduce_run({"compressed_bytes": comp, "samples": sh.reads * n, "errors": 0, "chunks": sh.reads},
                        0.5 + rank)
    q.put((rank, sh.global_ids(), tot, t))
    dist.destroy_process_group()


def test_two_rank_shard_and_reduce():
    world, reads, n = 2, 6, 3000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, reads, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ids = sorted(i for _, g, _, _ in res for i in g)
    assert ids == list(range(world * reads))  # round-robin shards partition the read set
    import _oracle as O

    want = sum(len(O.c5_compress(O.synth_read(g, n))[1]) for g in range(world * reads))
    for _, _, tot, t in res:
        assert tot["compressed_bytes"] == want
        assert tot["samples"] == world * reads * n and tot["chunks"] == world * reads
        assert t == 1.5  # max over ranks


def test_shard_validation():
    from rawnanoporesignalcompression_amd.shard import shard_reads

    s = shard_reads(4, 1, 3)
    assert s.global_ids() == [1, 4, 7, 10]
    with pytest.raises(ValueError):
        shard_reads(4, 3, 3)
