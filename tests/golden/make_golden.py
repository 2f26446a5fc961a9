"""Regenerate the committed fixtures under tests/golden/ (run in the build container, where the
reference tree is mounted read-only at /root/reference).

Inputs are data only:
  * the `signal` / `samples` columns of the reference's own POD5 test fixture
    pod5/test_data/multi_fast5_zip_v3.pod5 (VBZ-compressed real nanopore signal, 22 chunks), read with
    pyarrow from the file's embedded Arrow IPC signal table;
  * synthetic reads from the checker's generator.
Expected outputs come from the oracle (oracle/pgn_oracle.c over libzstd 1.4.9).  The C5 split of every
fixture chunk is also produced by the reference's OWN svb16 code (oracle/_ref/libpgn_ref.so, compiled
verbatim from C5.hpp:27-277 by oracle/ref.mk): those digests are recorded as `ref_streams_sha256`
(after asserting the oracle's streams equal them) so the pin travels without the reference tree.

Usage: python tests/golden/make_golden.py [/path/to/multi_fast5_zip_v3.pod5]
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import _oracle as O  # noqa: E402

POD5 = "/root/reference/pod5/test_data/multi_fast5_zip_v3.pod5"

# sizes at the C5 / zstd thresholds: key/nibble tails, FCS sizes, cparam tiers
EDGE_SIZES = [0, 1, 2, 3, 4, 5, 7, 8, 63, 64, 255, 256, 257, 1023, 1024, 16384, 16385, 65791, 65792, 65793,
              102399, 102400]


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def read_signal_table(path: str):
    import pyarrow as pa
    import pyarrow.ipc as ipc

    raw = open(path, "rb").read()
    # the first embedded Arrow file of a combined POD5 is the signal table
    start = raw.index(b"ARROW1")
    end = raw.index(b"ARROW1", start + 6) + 6
    table = ipc.open_file(pa.BufferReader(raw[start:end])).read_all()
    blobs = [bytes(b) for b in table.column("signal").to_pylist()]
    counts = table.column("samples").to_pylist()
    read_ids = [bytes(r).hex() for r in table.column("read_id").to_pylist()]
    return blobs, counts, read_ids


def main(path: str = POD5) -> None:
    assert O.ref() is not None, "the reference check needs /root/reference (oracle/ref.mk)"
    blobs, counts, read_ids = read_signal_table(path)
    offs = np.cumsum([0] + [len(b) for b in blobs]).astype(np.int64)
    np.savez_compressed(os.path.join(HERE, "pod5_v3_signal.npz"),
                        vbz=np.frombuffer(b"".join(blobs), np.uint8), vbz_offsets=offs,
                        samples=np.array(counts, np.uint32))
    real = []
    tot_c5 = tot_vbz = tot_n = 0
    for i, (b, n) in enumerate(zip(blobs, counts)):
        rc, x = O.vbz_decompress(b, n)
        assert rc == 0
        vbz_again = O.vbz_compress(x)
        rc, c5, st = O.c5_compress(x)
        assert rc == 0
        rc2, back = O.c5_decompress(c5, n)
        assert rc2 == 0 and np.array_equal(back, x)
        ref_streams = O.ref_variant_streams("C5", x)
        assert ref_streams == O.variant_streams("C5", x), f"chunk {i}: oracle split differs from the reference"
        real.append({"ref_streams_sha256": [sha(b) for b in ref_streams], "chunk": i, "read_id": read_ids[i], "samples": n, "signal_sha256": sha(x.tobytes()),
                     "vbz_size": len(b), "vbz_reencode_identical": vbz_again == b,
                     "c5_size": len(c5), "c5_sha256": sha(c5), "streams": [int(v) for v in st]})
        tot_c5 += len(c5)
        tot_vbz += len(b)
        tot_n += n
    synth = []
    for r in range(6):
        x = O.synth_read(r, 100000)
        rc, c5, st = O.c5_compress(x)
        synth.append({"read": r, "samples": 100000, "signal_sha256": sha(x.tobytes()), "c5_size": len(c5),
                      "c5_sha256": sha(c5), "streams": [int(v) for v in st]})
    edges = []
    for n in EDGE_SIZES:
        x = O.synth_read(1000 + n, n)
        rc, c5, st = O.c5_compress(x)
        edges.append({"samples": n, "signal_sha256": sha(x.tobytes()), "status": rc,
                      "c5_size": len(c5), "c5_sha256": sha(c5)})
    # small byte-exact blobs kept whole (first two real chunks, a tiny synthetic read)
    keep = {}
    for i in (0, 1):
        rc, x = O.vbz_decompress(blobs[i], counts[i])
        keep[f"real{i}"] = O.c5_compress(x)[1]
    keep["synth_small"] = O.c5_compress(O.synth_read(7, 3000))[1]
    np.savez_compressed(os.path.join(HERE, "c5_blobs.npz"),
                        **{k: np.frombuffer(v, np.uint8) for k, v in keep.items()})
    doc = {
        "generator": "tests/golden/make_golden.py",
        "zstd_version": int(O.oracle().pgno_zstd_version()),
        "ref_pinned": {"c5_streams": True, "library": "oracle/_ref/libpgn_ref.so",
                       "recipe": "oracle/ref.mk (C5.hpp:27-277 compiled verbatim)"},
        "real": real,
        "real_totals": {"samples": tot_n, "c5_bits_per_sample": 8.0 * tot_c5 / tot_n,
                        "vbz_bits_per_sample": 8.0 * tot_vbz / tot_n},
        "synth": synth,
        "edge": edges,
    }
    with open(os.path.join(HERE, "c5_golden.json"), "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc["real_totals"]))


if __name__ == "__main__":
    main(*(sys.argv[1:2]))
