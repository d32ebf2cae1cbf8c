"""One-bracket promotion with tied losses straddling the k-th place (GPU box): wall time per call of the
size-policy path (which sends these to the GPU re-rank) and numpy's rule; run under rocprofv3 for the
kernels.    python tools/tie_latency.py [n] [reps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from hpbandster_amd import promote
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    dev = torch.device("cuda", 0)
    for digits in (1, 2, 3):
        x = np.round(np.random.RandomState(3).rand(n), digits)
        k = n // 3
        promote.advance_mask(x, k, device=dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            promote.advance_mask(x, k, device=dev)
        t = (time.perf_counter() - t0) / reps * 1e6
        t0 = time.perf_counter()
        for _ in range(reps):
            np.argsort(np.argsort(x)) < k
        tn = (time.perf_counter() - t0) / reps * 1e6
        print({"n": n, "distinct": int(np.unique(x).size), "advance_mask_us": round(t, 1), "numpy_us": round(tn, 1)},
              flush=True)


if __name__ == "__main__":
    main()
