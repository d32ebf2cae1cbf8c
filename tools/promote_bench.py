"""Microbenchmark of the SH promotion select kernel at config #5's shape (1e4 brackets x 1e3 configs)
against a same-traffic elementwise floor (torch: read 80 MB of f64, write 10 MB of bool)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpbandster_amd import _native as N  # noqa: E402
from hpbandster_amd import synthetic as S  # noqa: E402

dev = torch.device("cuda", 0)
B, n = 10000, 1000
L = N.lib()
losses = torch.from_numpy(S.make_bracket_losses(B, n).reshape(-1)).to(dev)
seg = torch.arange(B + 1, dtype=torch.int64, device=dev) * n
k = torch.full((B,), float(n // 3), dtype=torch.float64, device=dev)
adv = torch.empty(B * n, dtype=torch.uint8, device=dev)
nadv = torch.empty(B, dtype=torch.int64, device=dev)
sh = N.stream_handle(None, dev)


def sel():
    N.check(L.hbx_sh_promote(N.ptr(losses), N.ptr(seg), B, n, B * n, N.ptr(k), None, N.ptr(adv), N.ptr(nadv), None, 0,
                             sh))


def floor():
    torch.lt(losses, 0.333, out=adv.view(torch.bool))


REPS = int(os.environ.get("PB_REPS", "50"))
for name, fn in (("select", sel), ("floor_lt", floor)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / REPS
    print("%-9s %.4f ms  %.0f GB/s (9 B/config)" % (name, ms, B * n * 9 / ms / 1e6), flush=True)
ok = (nadv == n // 3).all().item()
print("counts ok", ok)
