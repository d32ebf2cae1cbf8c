"""Batched successive-halving promotion on the GPU (HB_iteration.py:149-190, 203-250).

``advance = argsort(argsort(losses)) < k`` per bracket, over the REVIEW (finite-loss) entries;
CRASHED entries (non-finite loss) never advance.  Many brackets are ranked in one launch
(a radix select of the k-th loss per bracket, one wave each), which is what config #5 of the
benchmark exercises.
"""

import threading

import numpy as np

from . import _native as N
from .kde import default_device


def promote_segments(loss, seg_off, k, device=None, stream=None, return_order=False):
    """loss: fp64 [N] (numpy or device tensor); seg_off: int64 [B+1]; k: per-bracket threshold [B].

    Returns a bool numpy mask [N]; with ``return_order`` the device tensors (advance u8, sorted
    positions i64, advancing count per bracket i64).
    """
    import torch
    L = N.lib()
    device = device or default_device()
    with N.on_device(device, stream):
        return _promote_segments(L, loss, seg_off, k, device, stream, return_order)


def _promote_segments(L, loss, seg_off, k, device, stream, return_order):
    import torch

    def dev(a, dt):
        if isinstance(a, np.ndarray) or not hasattr(a, "data_ptr"):
            return torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=dt))).to(device)
        return a

    loss_d = dev(loss, np.float64)
    seg_h = np.asarray(seg_off.cpu().numpy() if hasattr(seg_off, "cpu") else seg_off, dtype=np.int64)
    seg_d = dev(seg_h, np.int64)
    k_d = dev(np.asarray(k, dtype=np.float64), np.float64)
    B = seg_h.shape[0] - 1
    Ntot = int(loss_d.shape[0])
    max_seg = int(np.max(np.diff(seg_h))) if B > 0 else 0
    # the sorted order only on request: brackets <= 1024 then take the O(n) select (no scratch)
    order = torch.empty(Ntot, dtype=torch.int64, device=device) if return_order else None
    adv = torch.empty(Ntot, dtype=torch.uint8, device=device)
    nadv = torch.empty(max(B, 1), dtype=torch.int64, device=device)
    scratch, sb = None, 0
    if return_order or max_seg > 1024:
        sb = int(L.hbx_sort_scratch_bytes(Ntot))
        scratch = torch.empty(sb, dtype=torch.uint8, device=device)
    N.check(L.hbx_sh_promote(N.ptr(loss_d), N.ptr(seg_d), B, max_seg, Ntot, N.ptr(k_d), N.ptr(order), N.ptr(adv),
                             N.ptr(nadv), N.ptr(scratch), sb, N.stream_handle(stream, device)))
    if return_order:
        return adv, order, nadv
    return adv.cpu().numpy().astype(bool)


class _Staging(object):
    """Per-thread, per-device buffers of advance_mask: pinned host in/out and their device twins,
    grown on demand.  Every call synchronises its stream before returning, so a buffer is free again
    when the next call of the same thread starts."""

    def __init__(self, device):
        self.device = device
        self.cap = 0

    def get(self, n):
        import torch
        if n > self.cap:
            cap = max(1024, 1 << (int(n) - 1).bit_length())
            self.h_in = torch.empty(cap + 3, dtype=torch.float64, pin_memory=True)
            self.h_out = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
            self.d_in = torch.empty(cap + 3, dtype=torch.float64, device=self.device)
            self.d_out = torch.empty(cap, dtype=torch.uint8, device=self.device)
            self.cap = cap
        return self


_tls = threading.local()


def _staging(device):
    import torch
    key = str(torch.device(device))
    st = getattr(_tls, "staging", None)
    if st is None:
        st = _tls.staging = {}
    if key not in st:
        st[key] = _Staging(device)
    return st[key]


def advance_mask(losses, k, device=None, stream=None):
    """Single bracket: bool mask of the configurations that advance (HB_iteration.py:180-182).

    What SuccessiveHalving.process_results calls once per bracket: segment bounds, k and the losses
    travel in one pinned host->device copy, the select kernel runs, the mask comes back in one pinned
    copy, one stream synchronisation."""
    import torch
    losses = np.asarray(losses, dtype=np.float64).reshape(-1)
    n = losses.shape[0]
    if n == 0:
        return np.zeros(0, dtype=bool)
    if n > 1024:
        return promote_segments(losses, np.array([0, n], dtype=np.int64), [k], device=device, stream=stream)
    device = device or default_device()
    L = N.lib()
    with N.on_device(device, stream):
        st = _staging(device).get(n)
        hb = st.h_in.numpy()
        hb[:2].view(np.int64)[:] = (0, n)
        hb[2] = float(k)
        hb[3:3 + n] = losses
        cur = stream if stream is not None else torch.cuda.current_stream(device)
        st.d_in[:n + 3].copy_(st.h_in[:n + 3], non_blocking=True)
        base = st.d_in.data_ptr()
        N.check(L.hbx_sh_promote(base + 24, base, 1, n, n, base + 16, None, N.ptr(st.d_out), None, None, 0,
                                 cur.cuda_stream))
        st.h_out[:n].copy_(st.d_out[:n], non_blocking=True)
        cur.synchronize()
        return st.h_out[:n].numpy().astype(bool)
