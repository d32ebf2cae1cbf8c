"""Time hbx_seg_argsort on one segment of n losses (the BOHB refit split) for each kernel path."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpbandster_amd import _native as N  # noqa: E402

dev = torch.device("cuda:0")
L = N.lib()
for n in (1000, 10000, 60000):
    loss = torch.from_numpy(np.random.RandomState(1).rand(n)).to(dev)
    seg = torch.tensor([0, n], dtype=torch.int64, device=dev)
    order = torch.empty(n, dtype=torch.int64, device=dev)
    sb = int(L.hbx_sort_scratch_bytes(n))
    scr = torch.empty(sb, dtype=torch.uint8, device=dev)
    for env in ("1", "0"):
        os.environ["HBX_SORT_RANK"] = env
        os.environ["HBX_PROMOTE_WAVE"] = env
        f = lambda: N.call("hbx_seg_argsort", N.ptr(loss), N.ptr(seg), 1, n, n, N.ptr(order), N.ptr(scr), sb,  # noqa
                           N.stream_handle())
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            f()
        e1.record()
        torch.cuda.synchronize()
        ok = np.array_equal(order.cpu().numpy(), np.argsort(loss.cpu().numpy(), kind="stable"))
        print("n=%6d fast_paths=%s  %.1f us  ok=%s" % (n, env, e0.elapsed_time(e1) / 20 * 1e3, ok), flush=True)
