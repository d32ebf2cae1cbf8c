"""Diagnostic: acquisition over BOHB-sampled candidates at the bench model (config #3's KDEs).
Prints shortlist size, flags, timings and the distribution of the fp32 estimates."""
import time

import numpy as np
import torch

from hpbandster_amd import kde
from hpbandster_amd import synthetic as S

dc, du, lv, n = 24, 8, 4, 10000
X = S.make_observations(n, dc, du, lv)
L = S.make_losses(n)
dev = torch.device("cuda", 0)
pair = kde.fit_pair(X, L, S.var_type_string(dc, du), dc + du + 1, device=dev)
levels = np.array([0] * dc + [lv] * du)
for Nc in (1000, 100000, 1000000):
    c, _, _ = pair.good.sample(levels, 3.0, Nc, seed=1, counter_base=0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res, ll, lg = pair.acquire(c, logs=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    cl = np.log(1e-8)
    print("Nc=%d  %.2f ms  %r" % (Nc, dt * 1e3, res))
    print("   l>1e-8: %d  g>1e-8: %d  l nan: %d  g nan: %d  ll range [%.1f, %.1f]  lg range [%.1f, %.1f]" % (
        (ll > cl).sum(), (lg > cl).sum(), np.isnan(ll).sum(), np.isnan(lg).sum(), np.nanmin(ll), np.nanmax(ll),
        np.nanmin(lg), np.nanmax(lg)))
    cc = c.cpu().numpy()
    print("   cand range [%.3f, %.3f]  frac outside [0,1] %.3f" % (cc[:, :dc].min(), cc[:, :dc].max(),
                                                                  ((cc[:, :dc] < 0) | (cc[:, :dc] > 1)).mean()))
