"""Latency of the drop-in's ranking step, one bracket of n configurations (GPU box):
numpy's argsort(argsort) < k (the reference's rule), promote.advance_mask (the drop-in), and the bare
hbx_sh_advance_mapped call with every argument prepared (the native floor the Python wrapper adds to).

    python tools/promote_latency.py [n] [reps]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hpbandster_amd import _native as N
from hpbandster_amd import promote


def per_call(fn, reps):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    dev = torch.device("cuda", 0)
    losses = np.random.RandomState(3).rand(n)
    k = n // 3
    want = np.argsort(np.argsort(losses)) < k
    assert (promote.advance_mask(losses, k, device=dev) == want).all()
    host = per_call(lambda: np.argsort(np.argsort(losses)) < k, reps)
    drop = per_call(lambda: promote.advance_mask(losses, k, device=dev), reps)
    st = promote._staging(dev).get(n)
    stream = torch.cuda.current_stream(dev).cuda_stream
    mask = np.empty(n, dtype=np.bool_)
    fn = N.lib().hbx_sh_advance_mapped
    lp, mp = losses.ctypes.data, mask.ctypes.data

    def bare():
        st.seq += 1
        fn(lp, n, float(k), mp, st._ptrs[0], st._ptrs[1], st.done_addr, st.seq, st.scr_ptr, N.ORDER_NUMPY, stream)

    native = per_call(bare, reps)
    assert (mask == want).all()
    # the host side of the launch alone (no wait; the stream is drained once at the end)
    one = N.lib().hbx_sh_promote_one

    def launch():
        one(st._ptrs[0], n, float(k), st._ptrs[1], st.scr_ptr, N.ORDER_NUMPY, None, 0, stream)

    launch_us = per_call(launch, 200)
    torch.cuda.synchronize()
    # launch + stream synchronisation (no completion-word polling)
    sync_us = per_call(lambda: (launch(), torch.cuda.current_stream(dev).synchronize()), reps)
    print({"n": n, "reps": reps, "host_numpy_us": round(host, 2), "advance_mask_us": round(drop, 2),
           "native_call_us": round(native, 2), "launch_only_us": round(launch_us, 2),
           "launch_sync_us": round(sync_us, 2)})


if __name__ == "__main__":
    main()
