import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np, torch
import _oracle as O
from test_gpu_multiblock import _c5_signals
from rawnanoporesignalcompression_amd import PGNanoCodec
c = PGNanoCodec(0)
for name, x in _c5_signals().items():
    rc, ref, _ = O.c5_compress(x)
    if rc: continue
    try:
        y = c.decompress_signal(ref, sample_count=x.size); ok1 = np.array_equal(y, x)
    except Exception as e:
        ok1 = repr(e)[:60]
    blobs = torch.from_numpy(np.frombuffer(ref, np.uint8).copy()).cuda()
    cnt = torch.tensor([x.size], dtype=torch.int32).cuda()
    out, so, st = c.decompress_batch(blobs, torch.zeros(1, dtype=torch.int64).cuda(), torch.tensor([len(ref)]).cuda(), cnt)
    torch.cuda.synchronize()
    ok2 = int(st[0]) == 0 and np.array_equal(out.cpu().numpy()[:x.size], x)
    print(name, "per-chunk:", ok1, "batch:", ok2, int(st[0]), c.kernels(1))
