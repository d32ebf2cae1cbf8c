"""Batched successive-halving promotion on the GPU (HB_iteration.py:149-190, 203-250).

``advance = argsort(argsort(losses)) < k`` per bracket, over the REVIEW (finite-loss) entries;
CRASHED entries (non-finite loss) never advance.  Many brackets are ranked in one launch (a selection
of the k-th loss per bracket, one wave each), which is what config #5 of the benchmark exercises.

Tied losses: ``ties='numpy'`` (default) ranks them as the reference's ``np.argsort`` does -- numpy
1.26.4's unstable AVX-512 quicksort, restated on the device (``hbx_npsort.h``): brackets whose tied
losses straddle the k-th place are re-ranked in that order.  ``ties='stable'`` ranks them by position.
"""

import ctypes
import math
import threading

import numpy as np

from . import _native as N
from .kde import default_device


def promote_segments(loss, seg_off, k, device=None, stream=None, return_order=False, ties="numpy"):
    """loss: fp64 [N] (numpy or device tensor); seg_off: int64 [B+1]; k: per-bracket threshold [B].

    Returns a bool numpy mask [N]; with ``return_order`` the device tensors (advance u8, sorted
    positions i64, advancing count per bracket i64).
    """
    L = N.lib()
    device = device or default_device()
    with N.on_device(device, stream):
        return _promote_segments(L, loss, seg_off, k, device, stream, return_order, N.order_mode(ties))


def _promote_segments(L, loss, seg_off, k, device, stream, return_order, mode):
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
    # the sorted order only on request: brackets <= 1024 then take the O(n) select
    order = torch.empty(Ntot, dtype=torch.int64, device=device) if return_order else None
    adv = torch.empty(Ntot, dtype=torch.uint8, device=device)
    nadv = torch.empty(max(B, 1), dtype=torch.int64, device=device)
    sb = int(L.hbx_sh_promote_scratch_bytes(B, max_seg, Ntot, 1 if return_order else 0, mode))
    scratch = torch.empty(sb, dtype=torch.uint8, device=device) if sb > 0 else None
    N.check(L.hbx_sh_promote_ex(N.ptr(loss_d), N.ptr(seg_d), B, max_seg, Ntot, N.ptr(k_d), N.ptr(order), N.ptr(adv),
                                N.ptr(nadv), N.ptr(scratch), sb, mode, None, N.stream_handle(stream, device)))
    if return_order:
        return adv, order, nadv
    return adv.cpu().numpy().astype(bool)


class _Staging(object):
    """Per-thread, per-device buffers of advance_mask: device-mapped coherent host memory for the
    losses (in) and the mask (out) -- the kernel reads and writes them directly, no copies -- and the
    device scratch of the numpy-order re-rank, grown on demand.  Every call waits for its kernel's
    completion word before returning, so the buffers are free again when the next call of the same
    thread starts."""

    def __init__(self, device):
        self.device = device
        self.index = device.index
        self.cap = 0
        self._ptrs = []
        self.fn = N.lib().hbx_sh_advance_state
        # hbx_sh_advance_state's block: {pin, pout, done, scratch, order_mode, seq, device}; the native call
        # launches on `device` whatever device is current on the calling thread
        self.state = (ctypes.c_int64 * 7)()
        self.state[6] = self.index
        self.state_addr = ctypes.addressof(self.state)
        self.mode = None
        self.stream_of = _current_stream_fn()

    def get(self, n):
        import torch
        if n > self.cap:
            L = N.lib()
            cap = max(1024, 1 << (int(n) - 1).bit_length())
            self._release()
            pin, pout = ctypes.c_void_p(), ctypes.c_void_p()
            N.check(L.hbx_host_alloc(8 * cap, ctypes.addressof(pin)))  # portable: mapped for every device
            N.check(L.hbx_host_alloc(cap + 64, ctypes.addressof(pout)))
            self._ptrs = [pin.value, pout.value]
            self.pin, self.pout = pin.value, pout.value
            # numpy views of the mapped buffers: the call fills / reads them in place (an ndarray's
            # .ctypes.data costs ~1 us per array, as much as the copies it would feed)
            self.pin_v = np.frombuffer((ctypes.c_double * cap).from_address(self.pin), dtype=np.float64)
            self.pout_v = np.frombuffer((ctypes.c_uint8 * cap).from_address(self.pout), dtype=np.bool_)
            # the completion word the kernel stores last (after the mask, system scope)
            self.done_addr = pout.value + cap
            ctypes.c_int32.from_address(self.done_addr).value = 0
            with torch.cuda.device(self.device):
                self.scratch = torch.empty(4 * cap, dtype=torch.int32, device=self.device)
            self.scr_ptr = self.scratch.data_ptr()
            self.cap = cap
            self.state[0], self.state[1], self.state[2], self.state[3] = self.pin, self.pout, self.done_addr, \
                self.scr_ptr
        return self

    def _release(self):
        for p in self._ptrs:
            N.lib().hbx_host_free(p)
        self._ptrs = []

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass


_tls = threading.local()


def _staging(device):
    """The calling thread's staging of `device` (None: torch's current device)."""
    st = getattr(_tls, "staging", None)
    if st is None:
        st = _tls.staging = {}
    if device is None:
        import torch
        device = torch.cuda.current_device()
    s = st.get(device)
    if s is None:
        import torch
        if not torch.cuda.is_available():
            raise N.HbxError("hpbandster_amd needs a ROCm GPU (torch.cuda.is_available() is False); "
                             "the engine has no CPU path")
        dev = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        key = str(dev)
        s = st.get(key)
        if s is None:
            s = st[key] = _Staging(dev)
        st[device] = s
    return s


def _current_stream_fn():
    import torch
    raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)  # the handle without a Stream object
    if raw is not None:
        return raw
    return lambda idx: torch.cuda.current_stream(idx).cuda_stream


_MODES = {"numpy": N.ORDER_NUMPY, "stable": N.ORDER_STABLE, N.ORDER_NUMPY: N.ORDER_NUMPY,
          N.ORDER_STABLE: N.ORDER_STABLE}

# one-bracket size policy (bench ``promote_dropin``, profiles/r04/promote_latency.txt): up to HOST_MAX
# configurations a bracket whose k-th and (k+1)-th smallest losses differ is ranked on the host -- every
# sort gives the same first k then, so the mask is the reference's bit for bit -- because one kernel round
# trip (launch, PCIe reads of the losses, the completion word: >= 8.3 us) costs more than numpy's sort of
# a few hundred values (n = 81: 1.9 us against 12.0 us for the GPU round trip and 2.5 us for the reference's
# argsort(argsort); n = 1000: 3.8 / 12.6 / 12.2 us; n = 4096: 7.2 us against 291 us through the sorting
# kernels brackets > 1024 take).  Brackets with a tie straddling the k-th place (numpy 1.26.4's unstable
# order decides them -- this process's numpy orders 65 of 206 recorded arrays differently) and non-finite
# losses are ranked on the host too, by libhbx's host restatement of that sort (hbx_sh_advance_host);
# larger brackets go to the GPU.
HOST_MAX = 1 << 16
_SORT_MAX = 256  # below: one argsort; above: np.partition (O(n))


def _threshold(k, n):
    """Number of ranks r in [0, n) with r < k (HB_iteration.py:180: ``ranks < k``; k may be fractional,
    SuccessiveResampling's num_configs * (1 - rate)); NaN or k <= 0: none."""
    if not k > 0:
        return 0
    return n if k >= n else int(math.ceil(k))


def _host_rank(losses, kk, n):
    """The mask of a tie-free bracket on the host, or None when the GPU must rank it (a tie across the
    k-th place, a non-finite loss)."""
    if kk == 0 or kk == n:
        if not math.isfinite(float(losses.sum())):
            return None
        return np.full(n, kk == n, dtype=bool)
    if n <= _SORT_MAX:
        o = losses.argsort()
        a, b = losses[o[kk - 1]], losses[o[kk]]
        # finite: argsort puts -inf first and +inf / NaN last
        if not (a < b and math.isfinite(losses[o[0]]) and math.isfinite(losses[o[n - 1]])):
            return None
        m = np.zeros(n, dtype=bool)
        m[o[:kk]] = True
        return m
    p = np.partition(losses, (kk - 1, kk))
    a, b = p[kk - 1], p[kk]
    if not (a < b and math.isfinite(float(losses.sum()))):
        return None
    return losses <= a


def _host_rank_ordered(losses, kk, n, ties):
    """A bracket whose tied losses straddle the k-th place, or with non-finite losses, on the host in the
    requested tie order: numpy 1.26.4's (hbx_sh_advance_host, the x86-simd-sort / introsort restatement in
    libhbx's host code) or by position.  As on the device, non-finite losses are CRASHED runs: never
    ranked, never advanced, and the first min(k, finite count) of the finite losses' argsort advance."""
    fin = None
    if not math.isfinite(float(losses.sum())):
        fin = np.isfinite(losses)
        sub = np.ascontiguousarray(losses[fin])
        kk = min(kk, sub.shape[0])
    else:
        sub = losses if losses.flags.c_contiguous else np.ascontiguousarray(losses)
    m = sub.shape[0]
    if kk == 0 or kk == m:
        adv = np.full(m, kk == m and m > 0, dtype=bool)
    else:
        mode = _MODES.get(ties)
        if mode is None:
            mode = N.order_mode(ties)
        if mode == N.ORDER_STABLE:
            adv = np.zeros(m, dtype=bool)
            adv[np.argsort(sub, kind="stable")[:kk]] = True
        else:
            hb = getattr(_tls, "host", None)
            if hb is None or hb[0] < m:  # per-thread output and scratch, their addresses taken once
                cap = max(1024, 1 << (m - 1).bit_length())
                a, sc = np.empty(cap, dtype=np.bool_), np.empty(cap, dtype=np.int64)
                hb = _tls.host = (cap, a, sc, a.ctypes.data, sc.ctypes.data, N.lib().hbx_sh_advance_host)
            rc = hb[5](sub.ctypes.data, m, kk, hb[3], hb[4])
            if rc:
                N.check(rc)
            adv = hb[1][:m].copy()
    if fin is None:
        return adv
    out = np.zeros(n, dtype=bool)
    out[fin] = adv
    return out


def advance_mask(losses, k, device=None, stream=None, ties="numpy", policy="auto"):
    """Single bracket: bool mask of the configurations that advance (HB_iteration.py:180-182).

    What SuccessiveHalving.process_results calls once per bracket.  ``policy='auto'``: brackets of at most
    HOST_MAX configurations are ranked on the host -- tie-free ones by numpy's argsort / partition (any sort
    gives the same first k), ones with tied losses across the k-th place or non-finite losses by libhbx's
    host restatement of numpy 1.26.4's sort (hbx_sh_advance_host) -- because one GPU round trip costs more
    than the sort.  Larger brackets, and everything with ``policy='gpu'``, go to the GPU: the losses are
    copied into device-mapped host memory, ONE host call into libhbx (hbx_sh_advance_state) launches the
    one-kernel promotion (the selection, and the numpy-order re-rank when tied losses straddle the k-th
    place), spins on the kernel's completion word (stored last) instead of synchronising the stream, and the
    mask is copied out."""
    if type(losses) is not np.ndarray or losses.ndim != 1 or losses.dtype != np.float64:
        losses = np.asarray(losses, dtype=np.float64).reshape(-1)
    n = losses.shape[0]
    if n == 0:
        return np.zeros(0, dtype=bool)
    if policy == "auto" and n <= HOST_MAX:
        kk = _threshold(k, n)
        m = _host_rank(losses, kk, n)
        if m is None:
            m = _host_rank_ordered(losses, kk, n, ties)
        return m
    elif policy not in ("auto", "gpu"):
        raise ValueError("policy must be 'auto' or 'gpu'")
    if n > 1024:
        return promote_segments(losses, np.array([0, n], dtype=np.int64), [k], device=device, stream=stream,
                                ties=ties)
    mode = _MODES.get(ties)
    if mode is None:
        mode = N.order_mode(ties)
    st = _staging(device).get(n)
    h = stream.cuda_stream if stream is not None else st.stream_of(st.index)
    if mode != st.mode:
        st.state[4] = st.mode = mode
    st.pin_v[:n] = losses  # straight into the mapped buffer the kernel reads
    rc = st.fn(st.state_addr, n, float(k), h)  # the sequence number advances in the state block
    if rc:
        N.check(rc)
    return st.pout_v[:n].copy()  # the mask, out of the mapped buffer the kernel wrote
