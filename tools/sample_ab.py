"""Dump and time GPU sampler draws (D = 32, 1e6 candidates, and odd / wide / small shapes) for an A/B
of two builds of libhbx.so (HBX_LIB_PATH):  python tools/sample_ab.py <tag>  -> gpurun_out/sample_<tag>.npz"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpbandster_amd import kde  # noqa: E402
from hpbandster_amd import synthetic as S  # noqa: E402

dev = torch.device("cuda", 0)
out = {}
for (dc, du, nobs, nc) in [(24, 8, 10000, 1_000_000), (5, 2, 300, 1001), (3, 0, 50, 77), (200, 40, 400, 3000)]:
    X = S.make_observations(nobs, dc, du, 4)
    loss = S.make_losses(nobs)
    pair = kde.fit_pair(X, loss, S.var_type_string(dc, du), dc + du + 1, device=dev)
    g = pair.good
    lv = [0] * dc + [4] * du
    for table in (False, True):
        c, dat, err = g.sample(lv, 3.0, nc, seed=1234, counter_base=7, table=table)
        torch.cuda.synchronize()
        tag = "d%d_%d_t%d" % (dc + du, nc, table)
        out[tag] = c.cpu().numpy()
        out[tag + "_datum"] = dat.cpu().numpy()
        out[tag + "_err"] = err.cpu().numpy()
    if nc >= 1_000_000:
        for _ in range(3):
            g.sample(lv, 3.0, nc, seed=1, counter_base=0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for r in range(20):
            g.sample(lv, 3.0, nc, seed=r, counter_base=0)
        torch.cuda.synchronize()
        print("%s: %.4f ms per 1e6 x %d draw" % (sys.argv[1], (time.perf_counter() - t0) / 20 * 1e3, dc + du))
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/sample_%s.npz" % sys.argv[1], **out)
