"""Stage stamps of the one-bracket numpy-order re-rank (needs the NPS_TIMING build:
HBX_LIB_PATH=ab/libhbx_nps.so python tools/nps_stamps.py): us from the kernel's staging start."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from hpbandster_amd import _native as N
    from hpbandster_amd import promote
    dev = torch.device("cuda", 0)
    L = N.lib()
    L.hbx_debug_nps.argtypes = [ctypes.c_void_p]
    L.hbx_debug_nps.restype = ctypes.c_int
    for digits in (1, 2, 3):
        x = np.round(np.random.RandomState(3).rand(1000), digits)
        promote.advance_mask(x, 333, device=dev)
        buf = (ctypes.c_uint64 * 64)()
        L.hbx_debug_nps(ctypes.addressof(buf))
        v = np.array(buf[:], dtype=np.float64)
        t0 = v[40]
        rel = {k: round((v[k] - t0) / 100.0, 2) for k in list(range(0, 20)) + [40, 41, 42, 63] if v[k] >= t0 > 0}
        print({"distinct": int(np.unique(x).size), "stamps_us": rel}, flush=True)


if __name__ == "__main__":
    main()
