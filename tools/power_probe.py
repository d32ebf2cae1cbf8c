"""Keep the bench's scoring launch busy for a few seconds (for power / clock sampling with rocm-smi
or amd-smi beside it): python tools/power_probe.py [seconds]."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpbandster_amd import kde  # noqa: E402
from hpbandster_amd import synthetic as S  # noqa: E402

dev = torch.device("cuda", 0)
X = S.make_observations(10000, 24, 8, 4)
pair = kde.fit_pair(X, S.make_losses(10000), S.var_type_string(24, 8), 33, device=dev)
C = torch.from_numpy(S.make_candidates(1000000, 24, 8, 4)).to(dev)
sec = float(sys.argv[1]) if len(sys.argv) > 1 else 6.0
pair.acquire(C)
torch.cuda.synchronize()
t0, n = time.time(), 0
while time.time() - t0 < sec:
    for _ in range(20):
        pair.acquire(C)
    torch.cuda.synchronize()
    n += 20
dt = time.time() - t0
print("acquisitions %d in %.2f s: %.3f ms each" % (n, dt, dt / n * 1e3), flush=True)
