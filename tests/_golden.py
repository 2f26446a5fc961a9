"""Loaders for the committed fixtures in tests/golden/ (see make_golden.py)."""
import json
import os

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden():
    with open(os.path.join(HERE, "c5_golden.json")) as f:
        return json.load(f)


def real_vbz_chunks():
    z = np.load(os.path.join(HERE, "pod5_v3_signal.npz"))
    v, o, n = z["vbz"], z["vbz_offsets"], z["samples"]
    return [(v[o[i]:o[i + 1]].tobytes(), int(n[i])) for i in range(len(n))]


def c5_blobs():
    z = np.load(os.path.join(HERE, "c5_blobs.npz"))
    return {k: z[k].tobytes() for k in z.files}
