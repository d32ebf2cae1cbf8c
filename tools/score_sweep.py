"""Scoring-kernel sweep on the GPU: ms per hbx_kde_logpdf launch vs observation count at fixed Nc.

The intercept of the fit is the per-launch fixed cost (candidate prologue, pipeline fill, tail),
the slope the per-64-observation-chunk cost.  python tools/score_sweep.py [--nc 1000000]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpbandster_amd import kde  # noqa: E402
from hpbandster_amd import synthetic as S  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--nc", type=int, default=1_000_000)
ap.add_argument("--dc", type=int, default=24)
ap.add_argument("--du", type=int, default=8)
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
dev = torch.device("cuda", 0)
vt = S.var_type_string(a.dc, a.du)
X = S.make_observations(10000, a.dc, a.du, 4)
L = S.make_losses(10000)
pair = kde.fit_pair(X, L, vt, a.dc + a.du + 1, device=dev)
bad = pair.bad
C = torch.from_numpy(S.make_candidates(a.nc, a.dc, a.du, 4)).to(dev)
rows_all = bad.rows_dev.cpu().numpy()
out = []
for n in (64, 256, 1024, 1500, 4096, 8500):
    k = kde.DeviceKDE(bad.X_dev, torch.from_numpy(rows_all[:n].copy()).to(dev), vt, bad.bw, bad.nlev,
                      X[rows_all[:n]])
    k.logpdf_est(C[:1024])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    from hpbandster_amd import _native as N
    est = torch.empty((a.nc, 4), dtype=torch.float32, device=dev)
    Lb = N.lib()
    ts = []
    for r in range(a.reps):
        e0.record()
        N.check(Lb.hbx_kde_logpdf(N.ptr(C), a.nc, k.k_vars, N.ptr(k.params), N.ptr(k.table), k.dc_pad, k.du_pad,
                                  k.variant, N.ptr(est), N.stream_handle()))
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = float(np.median(ts))
    out.append({"n": n, "ms": ms, "pairs_per_s": a.nc * n / ms * 1e3})
    print(json.dumps(out[-1]), flush=True)
ns = np.array([o["n"] for o in out], float)
ms = np.array([o["ms"] for o in out])
A = np.vstack([np.ceil(ns / 64), np.ones_like(ns)]).T
slope, icpt = np.linalg.lstsq(A, ms, rcond=None)[0]
print(json.dumps({"ms_per_chunk": slope, "intercept_ms": icpt,
                  "marginal_pairs_per_s": a.nc * 64 / slope * 1e3}))
