"""Fixed cost of one acquisition beyond its scoring work (GPU box, via gpurun):
    python tools/host_path.py [--reps 400]
For config #2 (1e5 x 1e3, D = 8) and a 64-candidate get_config against config #3's model: wall time per
synchronous acquisition through the drop-in (KDEPair.acquire), through the bare native call with every
argument prepared (hbx_kde_acquire_bound), the scoring launch alone (its own start/end stamps), and the
floor of any one-launch round trip (hbx_fetch of 8 bytes)."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def per_call(fn, reps):
    for _ in range(10):
        fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps * 1e6


def measure(pair, C, reps):
    import ctypes
    import torch
    from hpbandster_amd import _native as N
    from hpbandster_amd import kde
    L = N.lib()
    dev = pair.good.device
    Nc = int(C.shape[0])
    ws = torch.empty(pair.workspace_bytes(Nc), dtype=torch.uint8, device=dev)
    drop = per_call(lambda: pair.acquire(C, workspace=ws), reps)
    rec = ctypes.create_string_buffer(64)
    args = (pair._bound, C.data_ptr(), Nc, 0, ws.data_ptr(), ws.numel(), None, None, N.stream_handle(None, dev),
            ctypes.addressof(rec), None)
    fn = L.hbx_kde_acquire_bound
    native = per_call(lambda: fn(*args), reps)
    ev = kde.ScoreEvents()
    pair.acquire(C, workspace=ws, events=ev)
    ms = []
    for _ in range(50):
        pair.acquire(C, workspace=ws, events=ev)
        ms.append(sum(ev.elapsed_ms(True)))
    src = torch.zeros(2, dtype=torch.float64, device=dev)
    dst = np.zeros(2)
    fetch = L.hbx_fetch
    sh = N.stream_handle(None, dev)
    floor = per_call(lambda: fetch(dst.ctypes.data, src.data_ptr(), 8, sh), reps)
    return {"candidates": Nc, "obs": pair.good.nobs + pair.bad.nobs, "dropin_us": drop, "native_us": native,
            "scoring_launch_us": float(np.median(ms)) * 1e3, "fetch8_floor_us": floor,
            "dropin_minus_scoring_us": drop - float(np.median(ms)) * 1e3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=400)
    a = ap.parse_args()
    import torch
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    dev = torch.device("cuda", 0)
    out = {}
    variants = [v for v in os.environ.get("HOST_PATH_AB", "").split(",") if v]  # e.g. HBX_RESCUE_PASS=1
    X = S.make_observations(1000, 8, 0, 0)
    pair = kde.fit_pair(X, S.make_losses(1000), S.var_type_string(8, 0), 9, device=dev)
    C = torch.from_numpy(S.make_candidates(100_000, 8, 0, 0)).to(dev)
    out["config2"] = measure(pair, C, a.reps)
    for v in variants:
        k, val = v.split("=")
        old = os.environ.get(k)
        os.environ[k] = val
        out["config2_" + v] = measure(pair, C, a.reps)
        os.environ.pop(k) if old is None else os.environ.__setitem__(k, old)
    X = S.make_observations(10000, 24, 8, 4)
    pair = kde.fit_pair(X, S.make_losses(10000), S.var_type_string(24, 8), 33, device=dev)
    C = torch.from_numpy(S.make_candidates(64, 24, 8, 4)).to(dev)
    out["get_config_64"] = measure(pair, C, a.reps)
    C = torch.from_numpy(S.make_candidates(1000000, 24, 8, 4)).to(dev)
    out["config3"] = measure(pair, C, 40)
    for v in variants:
        k, val = v.split("=")
        old = os.environ.get(k)
        os.environ[k] = val
        out["config3_" + v] = measure(pair, C, 40)
        os.environ.pop(k) if old is None else os.environ.__setitem__(k, old)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
