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


# ---- bench.py's own orchestration under gloo (CPU stand-in codec) ------------------------------
def _bench_worker(rank, world, port, argv, q):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    import torch
    import torch.distributed as dist

    import bench
    from _cpu_codec import CpuCodec

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    args = bench.parse(argv)
    line = bench.run_rank(args, rank, world, rank, CpuCodec(), torch, dist, device="cpu", cuda=False)
    q.put((rank, line))
    dist.destroy_process_group()


def _run_bench_ranks(world, argv):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, argv, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_bench_rank_body_weak_scaling_two_ranks():
    """bench.run_rank on two gloo ranks: round-robin shards, barriers, SUM/MAX reduction, the line."""
    import _oracle as O

    reads, n = 3, 2000
    res = _run_bench_ranks(2, ["--gpus", "2", "--reads", str(reads), "--samples", str(n), "--steps", "1",
                               "--warmup", "0", "--no-side", "--no-cpu-baseline"])
    assert res[1] is None
    line = res[0]
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and line["round_trip_ok"]
    assert line["config"]["global_reads"] == 2 * reads
    want = sum(len(O.c5_compress(O.synth_read(g, n))[1]) for g in range(2 * reads))
    assert line["compressed_bytes"] == want
    assert line["value"] > 0 and line["roofline"]["traffic"] is None


def test_bench_rank_body_strong_scaling_batches():
    """--global-reads: a fixed read set split round-robin over the ranks, in batches of DISTINCT reads:
    the reported compressed bytes are those of every one of the G reads (measured, not extrapolated)."""
    import _oracle as O

    reads_total, n = 7, 1500
    res = _run_bench_ranks(2, ["--global-reads", str(reads_total), "--reads", "2", "--samples", str(n),
                               "--steps", "1", "--warmup", "0", "--no-side", "--no-cpu-baseline"])
    line = res[0]
    assert line["scaling"] == "strong" and line["round_trip_ok"]
    assert line["config"]["global_reads"] == reads_total
    assert line["config"]["reads_per_gpu"] == 4  # rank 0 owns reads 0, 2, 4, 6
    want = sum(len(O.c5_compress(O.synth_read(g, n))[1]) for g in range(reads_total))
    assert line["compressed_bytes"] == want
    # the same read set held resident (one batch per rank): same bytes
    res1 = _run_bench_ranks(2, ["--global-reads", str(reads_total), "--samples", str(n), "--steps", "1",
                                "--warmup", "0", "--no-side", "--no-cpu-baseline"])
    assert res1[0]["compressed_bytes"] == want and "resident" in res1[0]["config"]["workload"]


def test_rank_batches_partition():
    import bench

    for G, world, B in [(1_000_000, 8, 100_000), (1_000_000, 1, 100_000), (7, 3, 2), (5, 8, 4)]:
        args = bench.parse(["--global-reads", str(G), "--reads", str(B)])
        tot = 0
        for r in range(world):
            mine, batches, scaling = bench.rank_batches(args, r, world)
            assert scaling == "strong" and sum(batches) == mine and all(0 < b <= B for b in batches)
            assert mine == len(range(r, G, world))
            tot += mine
        assert tot == G
    mine, batches, scaling = bench.rank_batches(bench.parse([]), 0, 4)
    assert (mine, batches, scaling) == (100_000, [100_000], "weak")
    # configs[3] at 8 GPUs: a rank's 125,000 reads (75 GB at 6 B/sample) stay resident in one batch
    assert bench.rank_batches(bench.parse(["--global-reads", "1000000"]), 3, 8) == (125_000, [125_000], "strong")
    mine, batches, _ = bench.rank_batches(bench.parse(["--global-reads", "1000000"]), 0, 1)
    assert mine == 1_000_000 and len(batches) == 4 and max(batches) <= 333_333


def test_launcher_gives_each_rank_torchrun_env(tmp_path):
    """bench.py --gpus N outside torchrun: N worker processes with RANK/LOCAL_RANK/WORLD_SIZE and a
    127.0.0.1 rendezvous; a failing rank makes the launch fail."""
    import json

    import bench

    probe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_rank_probe.py")
    assert bench.launch_workers(3, [str(tmp_path), "-1"], script=probe, timeout=120) == 0
    envs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(3)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"] and [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    assert {e["WORLD_SIZE"] for e in envs} == {"3"} and {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1
    assert bench.launch_workers(2, [str(tmp_path), "1"], script=probe, timeout=120) == 3


# ---- multi-rank POD5 transcode (pod5_file.transcode_pod5_ranks) under gloo ----------------------
def _oracle_part(f, batch_ids, dst, variant):
    """CPU stand-in for pgn_pod5_transcode_part: the oracle decodes VBZ and encodes C5 row by row."""
    import numpy as np

    import _oracle as O

    assert dst == "pgnano" and variant == "C5"
    t = f.read_batches(batch_ids)
    blobs = []
    for i in range(t.rows):
        rc, x = O.vbz_decompress(t.blob(i), int(t.samples[i]))
        assert rc == 0
        rc, blob, _ = O.c5_compress(x)
        assert rc == 0
        blobs.append(np.frombuffer(blob, np.uint8))
    offs = np.zeros(t.rows + 1, np.uint64)
    np.cumsum([b.size for b in blobs], out=offs[1:])
    data = np.concatenate(blobs) if blobs else np.empty(0, np.uint8)
    return 0, (offs, data), [t.rows, int(t.samples.sum()), int(t.offsets[-1]), int(offs[-1])], [1.0, 2.0]


def _failing_part(f, batch_ids, dst, variant):
    if batch_ids and batch_ids[0] == 1:
        return 11, "synthetic failure", None, None
    return _oracle_part(f, batch_ids, dst, variant)


def _raising_part(f, batch_ids, dst, variant):
    """A rank whose local phase raises before any collective (as a failing codec or open would)."""
    if batch_ids and batch_ids[0] == 1:
        raise RuntimeError("codec creation failed")
    return _oracle_part(f, batch_ids, dst, variant)


def _transcode_worker(rank, world, port, src, out, rpb, fail, q):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    import torch.distributed as dist

    from rawnanoporesignalcompression_amd import pod5_file as Pm

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if fail in ("write", "marker") and rank == 1:  # rank 1's positioned writes fail
            real = Pm._write_rows_at

            def broken(path, pos, sizes, runs, offs, data, marker=None):
                if fail == "write":
                    raise OSError(28, "No space left on device (injected)")
                return real(path, pos, sizes, runs, offs, data, bytes(16))  # not the laid-out file's marker

            Pm._write_rows_at = broken
        part = {False: _oracle_part, True: _failing_part, "raise": _raising_part, "write": _oracle_part,
                "marker": _oracle_part}[fail]
        st = Pm.transcode_pod5_ranks(src, out, "pgnano", "C5", rows_per_batch=rpb, _part=part)
        q.put((rank, "ok", st))
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        q.put((rank, "error", f"{type(e).__name__}: {e}"))
    dist.destroy_process_group()


def _run_transcode(world, src, out, rpb, fail=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_transcode_worker, args=(r, world, port, src, out, rpb, fail, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _unmarked(path):
    b = open(path, "rb").read()
    return b.replace(b[8:24], bytes(16))  # the section marker is random per file


@pytest.mark.parametrize("world,src_rpb", [(2, 3), (3, 4), (2, 100)])
def test_multi_rank_transcode_matches_single_rank(tmp_path, world, src_rpb):
    """Record batches shared round-robin over gloo ranks, gathered on rank 0: the file is the one a
    single rank writes from the same per-row blobs (byte for byte, section marker aside)."""
    import numpy as np

    from _golden import HERE as GOLDEN
    from rawnanoporesignalcompression_amd import pod5_file as Pm

    src = str(tmp_path / "src.pod5")
    with Pm.Pod5File(os.path.join(GOLDEN, "multi_fast5_zip_v3.pod5")) as f:
        Pm.write_pod5(src, f.signal_table(), source=f, rows_per_batch=src_rpb)  # several record batches
    out = str(tmp_path / "multi.pod5")
    res = _run_transcode(world, src, out, rpb=7)
    assert all(r[1] == "ok" for r in res), res
    with Pm.Pod5File(src) as f:
        assert f.batches == -(-22 // src_rpb)
        st, (offs, data), counts, _ = _oracle_part(f, list(range(f.batches)), "pgnano", "C5")
        t = f.signal_table()
        one = str(tmp_path / "one.pod5")
        Pm.write_pod5(one, Pm.SignalTable(t.read_ids, t.samples, offs, data, "pgnano"), source=f, rows_per_batch=7)
    assert _unmarked(out) == _unmarked(one)
    for _, _, stats in res:
        assert stats["rows"] == 22 and stats["samples"] == counts[1]
        assert stats["in_bytes"] == counts[2] and stats["out_bytes"] == counts[3]
        assert stats["decode_ms"] == 1.0 and stats["encode_ms"] == 2.0
    with Pm.Pod5File(out) as g:
        assert g.signal_type == "pgnano" and g.rows == 22 and g.batches == 4
        np.testing.assert_array_equal(g.signal_table().offsets, offs)


def test_multi_rank_transcode_failure_raises_everywhere(tmp_path):
    from _golden import HERE as GOLDEN
    from rawnanoporesignalcompression_amd import pod5_file as Pm

    src = str(tmp_path / "src.pod5")
    with Pm.Pod5File(os.path.join(GOLDEN, "multi_fast5_zip_v3.pod5")) as f:
        Pm.write_pod5(src, f.signal_table(), source=f, rows_per_batch=3)
    out = tmp_path / "never.pod5"
    res = _run_transcode(2, src, str(out), rpb=100, fail=True)
    assert [r[1] for r in res] == ["error", "error"]
    assert "synthetic failure" in res[1][2] and "rank 1 failed" in res[0][2]
    assert not out.exists()


def test_multi_rank_transcode_local_exception_reaches_every_rank(tmp_path):
    """An exception in one rank's local phase (before any collective) becomes its status: every rank
    raises instead of waiting in a collective the failed rank never joins."""
    from _golden import HERE as GOLDEN
    from rawnanoporesignalcompression_amd import pod5_file as Pm

    src = str(tmp_path / "src.pod5")
    with Pm.Pod5File(os.path.join(GOLDEN, "multi_fast5_zip_v3.pod5")) as f:
        Pm.write_pod5(src, f.signal_table(), source=f, rows_per_batch=3)
    out = tmp_path / "never.pod5"
    res = _run_transcode(2, src, str(out), rpb=100, fail="raise")
    assert [r[1] for r in res] == ["error", "error"]
    assert "codec creation failed" in res[1][2] and "rank 1 failed" in res[0][2]
    assert not out.exists()


@pytest.mark.parametrize("mode", ["write", "marker"])
def test_multi_rank_transcode_write_failure_leaves_no_file(tmp_path, mode):
    """A rank whose positioned writes fail (ENOSPC), or that finds another file than the one rank 0
    laid out (section marker): every rank raises, out_path keeps its old content and the temporary
    file is gone."""
    from _golden import HERE as GOLDEN
    from rawnanoporesignalcompression_amd import pod5_file as Pm

    src = str(tmp_path / "src.pod5")
    with Pm.Pod5File(os.path.join(GOLDEN, "multi_fast5_zip_v3.pod5")) as f:
        Pm.write_pod5(src, f.signal_table(), source=f, rows_per_batch=3)
    out = tmp_path / "old.pod5"
    out.write_bytes(b"an older file of that name")
    res = _run_transcode(2, src, str(out), rpb=100, fail=mode)
    assert [r[1] for r in res] == ["error", "error"], res
    assert ("injected" if mode == "write" else "section marker") in res[1][2]
    assert "another rank failed to write" in res[0][2]
    assert out.read_bytes() == b"an older file of that name"
    assert sorted(p.name for p in tmp_path.iterdir()) == ["old.pod5", "src.pod5"]


def test_multi_rank_transcode_replaces_an_old_file(tmp_path):
    from _golden import HERE as GOLDEN
    from rawnanoporesignalcompression_amd import pod5_file as Pm

    src = str(tmp_path / "src.pod5")
    with Pm.Pod5File(os.path.join(GOLDEN, "multi_fast5_zip_v3.pod5")) as f:
        Pm.write_pod5(src, f.signal_table(), source=f, rows_per_batch=3)
    out = tmp_path / "old.pod5"
    out.write_bytes(b"x" * 10_000_000)
    res = _run_transcode(2, src, str(out), rpb=100)
    assert all(r[1] == "ok" for r in res), res
    with Pm.Pod5File(str(out)) as g:
        assert g.signal_type == "pgnano" and g.rows == 22
    assert sorted(p.name for p in tmp_path.iterdir()) == ["old.pod5", "src.pod5"]


def test_multi_rank_transcode_missing_input_raises_everywhere(tmp_path):
    res = _run_transcode(2, str(tmp_path / "absent.pod5"), str(tmp_path / "o.pod5"), rpb=100)
    assert [r[1] for r in res] == ["error", "error"]
