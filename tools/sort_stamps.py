"""Phase stamps of the one-launch refit sort (GPU box; a SORT_STAMPS build of libhbx via HBX_LIB_PATH):
    HBX_LIB_PATH=tools/_pst/libhbx_sstamps.so python tools/sort_stamps.py [n]
Median shader-clock cycles per phase over 20 refits of n observations x 32 dims (one new row each)."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from hpbandster_amd import _native as N
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    dev = torch.device("cuda", 0)
    nobs = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    X = S.make_observations(nobs, 24, 8, 4)
    losses = S.make_losses(nobs)
    n0 = nobs - 21
    store = kde.ObservationStore(32, S.var_type_string(24, 8), device=dev, capacity=2 * nobs)
    store.add(X[:n0], losses[:n0])
    store.refit(33)
    L = N.lib()
    L.hbx_debug_sort_stamps.argtypes = [ctypes.c_void_p]
    buf = np.zeros(16, dtype=np.uint64)
    spans = {"append rows + metadata": (0, 1), "barrier": (1, 2), "wave sort (registers)": (2, 3),
             "runs to LDS + rank merge": (3, 4), "scatter by rank": (4, 5), "tie check": (5, 6), "total": (0, 6)}
    rows = []
    for r in range(20):
        store.add(X[n0 + r], losses[n0 + r])
        store.refit(33)
        torch.cuda.synchronize()
        L.hbx_debug_sort_stamps(buf.ctypes.data)
        rows.append([float(int(buf[b]) - int(buf[a])) for a, b in spans.values()])
    med = np.median(np.array(rows), axis=0)
    print(json.dumps({"n": nobs, "cycles": dict(zip(spans, [float(v) for v in med]))}))


if __name__ == "__main__":
    main()
