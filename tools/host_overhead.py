"""Host time of the pieces of one acquisition call (GPU box):  python tools/host_overhead.py
The drop-in's KDEPair.acquire Python wrapper vs the bare ctypes call with every argument prepared, the
on_device context, the stream handle, the record fetch and its parse -- microseconds per call."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def per_call(fn, reps, sync=None):
    fn()
    if sync:
        sync()
    tot = 0.0
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        tot += time.perf_counter() - t0
        if sync:
            sync()
    return tot / reps * 1e6


def main():
    import torch
    from hpbandster_amd import _native as N
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    dev = torch.device("cuda", 0)
    dc, du, lev = 24, 8, 4
    X = S.make_observations(10000, dc, du, lev)
    pair = kde.fit_pair(X, S.make_losses(10000), S.var_type_string(dc, du), dc + du + 1, device=dev)
    Nc = 100000  # a short acquisition: the host pieces, not the GPU, are measured
    C = torch.from_numpy(S.make_candidates(Nc, dc, du, lev)).to(dev)
    ws = torch.empty(pair.workspace_bytes(Nc), dtype=torch.uint8, device=dev)
    L = N.lib()
    sync = torch.cuda.synchronize
    sh = N.stream_handle(None, dev)
    args = (C.data_ptr(), Nc, C.shape[1], 0) + tuple(pair._kde_args) + (None, None, ws.data_ptr(), ws.numel(), None, sh)
    rv = pair.acquire(C, workspace=ws, sync=False)
    out = {
        "on_device_ctx": per_call(lambda: N.on_device(dev).__enter__().__exit__(None, None, None), 20000),
        "stream_handle": per_call(lambda: N.stream_handle(None, dev), 20000),
        "acquire_wrapper": per_call(lambda: pair.acquire(C, workspace=ws, sync=False), 300, sync),
        "acquire_ctypes_only": per_call(lambda: L.hbx_kde_acquire(*args), 300, sync),
        "fetch_bytes_idle": per_call(lambda: kde.fetch_bytes(rv), 2000),
        "parse": per_call(lambda: kde.AcqResult.from_bytes(kde.fetch_bytes(rv)), 2000),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
