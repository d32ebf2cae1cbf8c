"""Host-side cost of one acquisition call (config #3 shape): the Python + C-ABI enqueue time of
KDEPair.acquire(sync=False) and the record read-back, beside the whole step.  python tools/time_host.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpbandster_amd import kde  # noqa: E402
from hpbandster_amd import synthetic as S  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
X = S.make_observations(10000, 24, 8, 4)
L = S.make_losses(10000)
pair = kde.fit_pair(X, L, S.var_type_string(24, 8), 33, device=dev)
C = torch.from_numpy(S.make_candidates(1000000, 24, 8, 4)).to(dev)
ws = torch.empty(pair.workspace_bytes(C.shape[0]), dtype=torch.uint8, device=dev)
ev = kde.ScoreEvents()
for _ in range(3):
    kde.AcqResult.from_bytes(kde.fetch_bytes(pair.acquire(C, workspace=ws, sync=False, events=ev)))
torch.cuda.synchronize()
enq, fetch, tot = [], [], []
for _ in range(20):
    t0 = time.perf_counter()
    rv = pair.acquire(C, workspace=ws, sync=False, events=ev)
    t1 = time.perf_counter()
    r = kde.AcqResult.from_bytes(kde.fetch_bytes(rv))
    t2 = time.perf_counter()
    ev.elapsed_ms(True)
    t3 = time.perf_counter()
    enq.append(t1 - t0)
    fetch.append(t2 - t1)
    tot.append(t3 - t0)
print("enqueue %.1f us  wait+fetch %.1f us  step %.1f us  events %.1f us" % (
    np.median(enq) * 1e6, np.median(fetch) * 1e6, np.median(tot) * 1e6, np.median(np.array(tot) - np.array(enq) - np.array(fetch)) * 1e6))
import cProfile, pstats
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    rv = pair.acquire(C, workspace=ws, sync=False, events=ev)
    kde.fetch_bytes(rv)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(15)
