"""Where the wall time of one incremental BOHB refit goes (config #3's observation set: 1e4 x 32):
cProfile over repeated ObservationStore.refit calls.  python tools/time_refit.py [reps]"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpbandster_amd import kde  # noqa: E402
from hpbandster_amd import synthetic as S  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda", 0)
X = S.make_observations(10000 + reps + 1, 24, 8, 4)
L = S.make_losses(10000 + reps + 1)
vt = S.var_type_string(24, 8)
D = X.shape[1]
store = kde.ObservationStore(D, vt, device=dev, capacity=2 * X.shape[0])
store.add(X[:10000], L[:10000])
store.refit(D + 1)
torch.cuda.synchronize()
for r in range(5):  # warm
    store.refit(D + 1)
t0 = time.perf_counter()
for r in range(reps):
    store.add(X[10000 + r], L[10000 + r])
    store.refit(D + 1)
print("ms per refit %.3f" % ((time.perf_counter() - t0) / reps * 1e3))
pr = cProfile.Profile()
pr.enable()
for r in range(reps):
    store.refit(D + 1)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
