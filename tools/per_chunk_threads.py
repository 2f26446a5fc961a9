"""Per-chunk plugin calls from one thread and from N host threads on one context (bench.py's
per_chunk_plugin / per_chunk_plugin_threads side numbers): python tools/per_chunk_threads.py [N ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

import bench
from rawnanoporesignalcompression_amd import PGNanoCodec

c = PGNanoCodec(0)
print(json.dumps({"threads": 1, **bench.per_chunk_plugin(torch, c, 100000, 42)}), flush=True)
for nt in [int(a) for a in sys.argv[1:]] or [4, 8, 16]:
    print(json.dumps(bench.per_chunk_plugin_threads(torch, c, 100000, 42, nthreads=nt, nreads=100 * nt)), flush=True)
