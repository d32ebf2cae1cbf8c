"""Where the headline step's time goes beyond the scoring launch (GPU box, via gpurun):
    python tools/step_breakdown.py [--steps 30]
Per step of bench.py's config #3 acquisition: host time inside pair.acquire (Python + native enqueue),
host time fetching the 48-byte record (copy + synchronisation), the scoring launch (its own start/end
stamps) and the GPU span from the stream event before the call to the one after the final kernel."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    import torch
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    dev = torch.device("cuda", 0)
    dc, du, lev, nobs, Nc = 24, 8, 4, 10000, 1000000
    X = S.make_observations(nobs, dc, du, lev)
    losses = S.make_losses(nobs)
    pair = kde.fit_pair(X, losses, S.var_type_string(dc, du), dc + du + 1, device=dev)
    C = torch.from_numpy(S.make_candidates(Nc, dc, du, lev)).to(dev)
    ws = torch.empty(pair.workspace_bytes(Nc), dtype=torch.uint8, device=dev)
    ev = kde.ScoreEvents()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    rows = []
    for s in range(a.steps + 3):
        t0 = time.perf_counter()
        e0.record()
        rv = pair.acquire(C, workspace=ws, sync=False, events=ev)
        e1.record()
        t1 = time.perf_counter()
        r = kde.AcqResult.from_bytes(kde.fetch_bytes(rv))
        t2 = time.perf_counter()
        if s >= 3:
            rows.append((t1 - t0, t2 - t1, t2 - t0, ev.elapsed_ms(True)[0] * 1e-3, e0.elapsed_time(e1) * 1e-3))
    sync = []  # the drop-in's synchronous call: hbx_kde_acquire_bound (the record on the host in one call)
    for s in range(a.steps + 3):
        t0 = time.perf_counter()
        r2 = pair.acquire(C, workspace=ws, events=ev)
        if s >= 3:
            sync.append((time.perf_counter() - t0, ev.elapsed_ms(True)[0] * 1e-3))
    assert r2.index == r.index
    m = np.median(np.array(rows), axis=0) * 1e6
    ms = np.median(np.array(sync), axis=0) * 1e6
    out = {"steps": a.steps, "median_us": {"acquire_call_host": m[0], "fetch_host": m[1], "step_host": m[2],
                                           "scoring_launch": m[3], "gpu_span_call": m[4]},
           "winner": r.index}
    out["median_us"]["step_minus_scoring"] = m[2] - m[3]
    out["median_us"]["sync_call_host"] = ms[0]
    out["median_us"]["sync_call_minus_scoring"] = ms[0] - ms[1]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
