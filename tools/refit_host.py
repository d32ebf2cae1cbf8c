"""Host-side pieces of one BOHB refit (ObservationStore.refit at config #3's 1e4 x 32, or n x 32), GPU box:
    python tools/refit_host.py [n]
Wall time per refit (with timing events around it, and without), the native hbx_kde_refit_sync call's own
host time, and the stream time (events)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from hpbandster_amd import _native as N
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    dev = torch.device("cuda", 0)
    nobs = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    X = S.make_observations(nobs, 24, 8, 4)
    losses = S.make_losses(nobs)
    D = 32
    reps = 30
    n0 = X.shape[0] - 2 * reps - 1
    store = kde.ObservationStore(D, S.var_type_string(24, 8), device=dev, capacity=2 * X.shape[0])
    store.add(X[:n0], losses[:n0])
    store.refit(D + 1)
    torch.cuda.synchronize()
    L = N.lib()
    native = []
    orig = L.hbx_kde_refit_sync

    def timed(*a):
        t0 = time.perf_counter()
        rc = orig(*a)
        native.append(time.perf_counter() - t0)
        return rc

    L.hbx_kde_refit_sync = timed
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    wall, stream = [], []
    for r in range(reps):
        store.add(X[n0 + r], losses[n0 + r])
        t0 = time.perf_counter()
        e0.record()
        store.refit(D + 1)
        e1.record()
        e1.synchronize()
        wall.append(time.perf_counter() - t0)
        stream.append(e0.elapsed_time(e1) * 1e-3)
    L.hbx_kde_refit_sync = orig
    # the same refits without the timing events around them: the call's own wall time
    plain = []
    for r in range(reps):
        store.add(X[n0 + reps + r], losses[n0 + reps + r])
        t0 = time.perf_counter()
        store.refit(D + 1)
        plain.append(time.perf_counter() - t0)
    print(json.dumps({"wall_us": float(np.median(wall)) * 1e6, "wall_us_no_events": float(np.median(plain)) * 1e6,
                      "native_call_us": float(np.median(native)) * 1e6, "stream_us": float(np.median(stream)) * 1e6}))


if __name__ == "__main__":
    main()
