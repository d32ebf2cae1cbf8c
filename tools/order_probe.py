"""Does the ORDER of the observation table's rows change the scoring launch's time?  (GPU box, via gpurun)
    python tools/order_probe.py [--reps 20]
The same observations X (config #3: 10^4 x 24c+8u) and candidates, three loss vectors: random (the bench's),
losses increasing along a Morton curve of the first continuous dims, and along the sum of the continuous
dims.  The split (argsort of the losses) lays the table out in loss order, so consecutive table rows --
the matrix instructions' consecutive A operands -- are spatially close in the second and third case.
Same pairs, same candidates, same flop count; alternating launches, pair-launch medians."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def morton_key(U, bits=10):
    q = np.clip((U * (1 << bits)).astype(np.int64), 0, (1 << bits) - 1)
    key = np.zeros(len(U), dtype=np.int64)
    nd = U.shape[1]
    for b in range(bits - 1, -1, -1):
        for d in range(nd):
            key = (key << 1) | ((q[:, d] >> b) & 1)
    return key


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    dev = torch.device("cuda", 0)
    dc, du, lev, nobs, Nc = 24, 8, 4, 10000, 1000000
    X = S.make_observations(nobs, dc, du, lev)
    vt = S.var_type_string(dc, du)
    rnd = S.make_losses(nobs)
    rs = np.random.RandomState(3)
    U = X[:, :5]
    mort = np.argsort(np.argsort(morton_key((U - U.min(0)) / (np.ptp(U, 0) + 1e-12), bits=6))) + rs.rand(nobs) * 0.5
    lin = X[:, :dc].sum(1)
    cases = {"random": rnd, "morton5": mort.astype(np.float64), "sum": lin}
    pairs = {k: kde.fit_pair(X, v, vt, dc + du + 1, device=dev) for k, v in cases.items()}
    C = torch.from_numpy(S.make_candidates(Nc, dc, du, lev)).to(dev)
    ws = torch.empty(pairs["random"].workspace_bytes(Nc), dtype=torch.uint8, device=dev)
    ev = kde.ScoreEvents()
    t = {k: [] for k in cases}
    for k, p in pairs.items():
        p.acquire(C, workspace=ws, events=ev)
    for r in range(a.reps):
        for k, p in pairs.items():
            res = p.acquire(C, workspace=ws, events=ev)
            t[k].append(ev.elapsed_ms(True)[0])
    out = {k: {"median_ms": float(np.median(v)), "mean_ms": float(np.mean(v)), "nobs": [pairs[k].good.nobs,
                                                                                        pairs[k].bad.nobs]}
           for k, v in t.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
