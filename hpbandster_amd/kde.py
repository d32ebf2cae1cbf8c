"""Device-resident BOHB KDE models: fit (refit per budget), scoring and exact acquisition.

The arithmetic mirrors the reference path exactly:

* split:      bohb.py:220-237 -- argsort the losses, good = head n_good, bad = tail n_bad
* bandwidth:  statsmodels 0.12.2 _kernel_base.py:250-265 -- 1.06 * np.std(X, 0) * n**(-1/(4+D))
* levels:     statsmodels kernels.py:59-60 -- observed np.unique(column).size per categorical dim
* pdf:        statsmodels kernel_density.py:162-196 / _kernel_base.py:456-518 (gpke)
* selection:  bohb.py:129,149-152 -- max(1e-8, g)/max(l, 1e-8), strict '<', first index wins

Everything that touches observations x candidates runs in libhbx.so (HIP, gfx950).  The host
side does O(D) bookkeeping only: the BOHB size rule, the pow() factor of the bandwidth rule (so it
rounds exactly like the reference's Python pow), and the small parameter block upload.
"""

import math
import struct
import threading

import numpy as np

from . import _native as N

RESULT_FMT = "<qdfiiidd"  # AcqResult: index, score, rel, flags, shortlist, near, pdf_l, pdf_g
RESULT_BYTES = struct.calcsize(RESULT_FMT)
ACQ_OVERFLOW, ACQ_NEAR_TIE, ACQ_RESOLVED, ACQ_DOMAIN_ERR = 1, 2, 4, 8  # include/hbx.h HBX_ACQ_*


def _torch():
    import torch
    return torch


def default_device():
    torch = _torch()
    if not torch.cuda.is_available():
        raise N.HbxError("hpbandster_amd needs a ROCm GPU (torch.cuda.is_available() is False); "
                         "the engine has no CPU path")
    return torch.device("cuda", torch.cuda.current_device())


def var_type_codes(var_type):
    return np.array([0 if c == "c" else 1 for c in var_type], dtype=np.int32)


def bohb_split_sizes(n, min_points, top_n_percent=15):
    """bohb.py:224-225."""
    return (max(min_points, (top_n_percent * n) // 100),
            max(min_points, ((100 - top_n_percent) * n) // 100))


def bandwidth_factor(nobs, D):
    """n**(-1/(4+D)) exactly as SM:_kernel_base.py:265 evaluates it (Python int ** float)."""
    return int(nobs) ** (-1. / (4 + int(D)))


def scoring_bucket(vt):
    """(dc_pad, du_pad) of the fp32 scoring kernel for var-type codes vt, or (-1, -1): no bucket fits
    (> 64 continuous or > 32 categorical dims) and the KDE is exact-only -- every candidate is re-scored
    in fp64 (hbx_kde_acquire handles it; hbx_kde_logpdf has no estimate for it)."""
    dc, du = int((vt == 0).sum()), int((vt == 1).sum())
    dcp, dup, stride = np.zeros(1, np.int32), np.zeros(1, np.int32), np.zeros(1, np.int32)
    if N.lib().hbx_kde_bucket(dc, du, N.ptr(dcp), N.ptr(dup), N.ptr(stride)) != 0:
        return -1, -1
    return int(dcp[0]), int(dup[0])


_pinned_tls = threading.local()


def _record_buffer():
    """This thread's host buffer for one result record (hbx_kde_acquire_bound writes it)."""
    import ctypes
    b = getattr(_pinned_tls, "rec", None)
    if b is None:
        b = _pinned_tls.rec = ctypes.create_string_buffer(64)
    return b


def mapped_candidates(n, D):
    """This thread's device-mapped coherent host buffer of n x D float64 candidates (hbx_host_alloc: the host
    address is the device's), as a numpy array: the host sampler draws straight into it and the acquisition's
    kernels read it in place (KDEPair.acquire_mapped) -- no host-to-device copy per get_config.  Reused by
    every call of the thread (each acquisition on it is synchronous); grown on demand."""
    import ctypes
    nbytes = 8 * n * D
    b = getattr(_pinned_tls, "cands", None)
    if b is None or b[1] < nbytes:
        if b is not None:  # (no acquisition of this thread reads the old one any more: they are synchronous)
            N.check(N.lib().hbx_host_free(b[0]))
        cap = max(nbytes, 64 * 64 * 8)
        p = ctypes.c_void_p()
        N.check(N.lib().hbx_host_alloc(cap, ctypes.addressof(p)))
        b = _pinned_tls.cands = (p.value, cap)
    return np.ctypeslib.as_array((ctypes.c_double * (n * D)).from_address(b[0])).reshape(n, D)


def fetch_bytes(dev_bytes, stream=None):
    """Bytes of a small device uint8 tensor (a result record) on the host: one native call (hbx_fetch)
    copies them into a per-thread, per-device pinned buffer on ``stream`` (default: the tensor's
    device's current stream) and polls that stream to completion -- instead of a pageable copy, or a
    torch copy plus a blocking stream synchronisation (~25 us more per acquisition)."""
    torch = _torch()
    n = int(dev_bytes.numel())
    dev = dev_bytes.device
    cache = getattr(_pinned_tls, "bufs", None)
    if cache is None:
        cache = _pinned_tls.bufs = {}
    key = (dev.index, n > 4096)
    buf = cache.get(key)
    if buf is None or buf.numel() < n:
        buf = torch.empty(max(n, 4096), dtype=torch.uint8, pin_memory=True)
        cache[key] = buf
    if not dev_bytes.is_contiguous():
        raise N.HbxError("fetch_bytes: contiguous device bytes expected")
    # one native call: the copy into the pinned buffer, then the stream polled to completion
    N.check(N.lib().hbx_fetch(buf.data_ptr(), dev_bytes.data_ptr(), n, N.stream_handle(stream, dev)))
    return buf[:n].numpy().tobytes()


class AcqResult(object):
    """One acquisition's winner (include/hbx.h result record).  ``flags`` & ACQ_NEAR_TIE: other
    candidates' exact scores lie within the spread another numpy build's exp could cause (``rel``);
    ACQ_RESOLVED: with ties='process' the host re-scored that near set with this process's numpy
    (exact_host) and picked from it."""
    __slots__ = ("index", "score", "rel", "flags", "shortlist", "near", "pdf_l", "pdf_g")

    def __init__(self, index, score, pdf_l, pdf_g, shortlist, flags, rel=0.0, near=1):
        self.index, self.score, self.pdf_l, self.pdf_g = int(index), score, pdf_l, pdf_g
        self.shortlist, self.flags, self.rel, self.near = int(shortlist), int(flags), float(rel), int(near)

    @classmethod
    def from_bytes(cls, b):
        idx, score, rel, fl, sl, near, l, g = struct.unpack(RESULT_FMT, bytes(b))
        return cls(idx, score, l, g, sl, fl, rel, near)

    def __repr__(self):
        return "AcqResult(index=%d, score=%r, pdf_l=%r, pdf_g=%r, shortlist=%d, near=%d, flags=%d)" % (
            self.index, self.score, self.pdf_l, self.pdf_g, self.shortlist, self.near, self.flags)


def _rows_of(cands, idx):
    """Candidate rows idx (host numpy) of a host array or a device tensor."""
    idx = np.asarray(idx, dtype=np.int64)
    if isinstance(cands, np.ndarray):
        return np.asarray(cands, dtype=np.float64)[idx]
    torch = _torch()
    return cands[torch.from_numpy(idx).to(cands.device)].cpu().numpy()


class DeviceKDE(object):
    """One fitted KDE (good or bad) on the GPU, with the statsmodels surface BOHB reads.

    ``data``/``bw``/``nobs``/``var_type``/``k_vars`` match ``KDEMultivariate`` (bohb.py:126-139
    reads ``.data``, ``.bw`` and ``.pdf``); ``pdf`` evaluates the exact fp64 density on the GPU.
    """

    def __init__(self, X_dev, rows_dev, var_type, bw, nlev, data_host, stream=None, prepared=None, home=None):
        """Prepare a KDE for scoring with ``hbx_kde_prepare`` -- or, with ``prepared`` = (params, table,
        info) from ``hbx_kde_refit``, wrap an already prepared one (``home``: the stream it was prepared on).
        ``data_host``: the observation rows (n x D), or a pair (host rows, row indices) gathered on first use of
        ``.data``.  Work on another stream is ordered after the preparation first (``_order``)."""
        self.var_type = var_type
        self.k_vars = len(var_type)
        self.bw = np.asarray(bw, dtype=np.float64)
        self.nlev = np.asarray(nlev, dtype=np.int32)
        self._data = data_host
        self.nobs = int(rows_dev.shape[0])
        self.X_dev = X_dev
        self.rows_dev = rows_dev
        self.device = X_dev.device
        D = self.k_vars
        if prepared is None:
            torch = _torch()
            L = N.lib()
            vt = var_type_codes(var_type)
            dcp, dup = scoring_bucket(vt)
            with N.on_device(self.device, stream):
                self.params = torch.empty(int(L.hbx_kde_param_bytes()), dtype=torch.uint8, device=self.device)
                tf = int(L.hbx_kde_table_floats(self.nobs, dcp, dup))
                self.table = torch.empty(tf, dtype=torch.float32, device=self.device)
                info = np.zeros(8, dtype=np.int32)
                bw_c = np.ascontiguousarray(self.bw)
                nlev_c = np.ascontiguousarray(self.nlev)
                home = N.stream_handle(stream, self.device)
                N.check(L.hbx_kde_prepare(N.ptr(X_dev), D, N.ptr(rows_dev), self.nobs, N.ptr(vt), N.ptr(bw_c),
                                          N.ptr(nlev_c), N.ptr(self.params), N.ptr(self.table), self.table.numel(),
                                          N.ptr(info), home))
        else:
            self.params, self.table, info = prepared
        self._home = home        # the stream the parameter block and table were written on
        self._ordered = set()    # other streams already ordered after that
        self.variant, self.nan_all, unsupported, self.dc, self.du, self.nconst, self.dc_pad, self.du_pad = \
            info.tolist()
        self.has_neg, self.kc = self.variant & 1, (self.variant >> 1) & 7
        self.exact_only = bool((self.variant >> 5) & 1)
        if unsupported:
            raise N.HbxError("KDE bandwidth/level combination not modelled (bw=%r, nlev=%r)" % (self.bw, self.nlev))

    @property
    def data(self):
        """KDEMultivariate.data: this KDE's observations (host, n x D), in the split's row order."""
        if isinstance(self._data, tuple):
            src, idx = self._data
            self._data = src[idx]
        return self._data

    def _order(self, sh):
        """Order stream ``sh`` after this model's preparation when it is not the stream that prepared it (once per
        stream: hbx_stream_order, no host wait)."""
        h = self._home
        if h is None or sh == h or sh in self._ordered:
            return
        N.check(N.lib().hbx_stream_order(sh, h))
        self._ordered.add(sh)

    def pdf(self, data_predict=None, stream=None):
        """Exact fp64 pdf on the GPU (KDEMultivariate.pdf semantics, np.squeeze'd)."""
        torch = _torch()
        L = N.lib()
        if data_predict is None:
            pts = np.asarray(self.data, dtype=np.float64)
        else:
            pts = np.asarray(data_predict, dtype=np.float64)
            if pts.ndim <= 1:
                pts = pts.reshape(-1, self.k_vars) if pts.size != self.k_vars else pts.reshape(1, -1)
        pts = np.ascontiguousarray(pts.reshape(-1, self.k_vars))
        with N.on_device(self.device, stream):
            p_dev = torch.from_numpy(pts).to(self.device)
            out = torch.empty(pts.shape[0], dtype=torch.float64, device=self.device)
            sb = int(L.hbx_kde_pdf_scratch_bytes(self.nobs))
            scratch = torch.empty(sb, dtype=torch.uint8, device=self.device)
            sh = N.stream_handle(stream, self.device)
            self._order(sh)
            N.check(L.hbx_kde_pdf_exact(N.ptr(p_dev), pts.shape[0], self.k_vars, N.ptr(self.params),
                                        N.ptr(self.X_dev), N.ptr(self.rows_dev), self.nobs, N.ptr(out), N.ptr(scratch),
                                        sb, sh))
            return np.squeeze(out.cpu().numpy())

    def sample(self, levels, bw_factor, Nc, seed, counter_base, stream_id=0, stream=None, table=None, out=None):
        """BOHB's candidate rule around this (good) KDE's observations, on the GPU (bohb.py:133-147).

        ``levels``: per dim 0 (continuous) or the number of choices.  Candidate i draws from the
        Philox stream (seed, counter_base + i, stream_id).  Returns (cands [Nc, D] f64, datum [Nc] i64,
        domain_err [Nc] u8) device tensors (``out``: those three tensors to fill instead of new ones)."""
        with N.on_device(self.device, stream):
            return self._sample(levels, bw_factor, Nc, seed, counter_base, stream_id, stream, table, out)

    def _sample(self, levels, bw_factor, Nc, seed, counter_base, stream_id, stream, table, out=None):
        torch = _torch()
        L = N.lib()
        D = self.k_vars
        sh = N.stream_handle(stream, self.device)
        self._order(sh)
        # the bandwidths the sampler reads: the prepared parameter block's own fp64 bw[D] (bit-identical
        # to self.bw, which was read back from it) -- no upload per refit
        bw_ptr = N.ptr(self.params) + int(L.hbx_kde_param_bw_offset())
        lv = np.ascontiguousarray(np.asarray(levels, dtype=np.int32))
        if lv.shape != (D,):
            raise N.HbxError("levels must have %d entries" % D)
        key = lv.tobytes()
        if getattr(self, "_lv_key", None) != key:
            self._lv_dev, self._lv_key = _levels_on_device(key, lv, self.device), key
            self._tab = None
        Nc = int(Nc)
        if table is None:
            table = Nc >= 4 * self.nobs  # the Phi table pays off when draws outnumber (row, dim) pairs
        tab = None
        if table:
            if getattr(self, "_tab", None) is None:
                self._tab = torch.empty(int(L.hbx_kde_sample_table_bytes(self.nobs, D)) // 8, dtype=torch.float64,
                                        device=self.device)
                N.check(L.hbx_kde_sample_table(N.ptr(self.X_dev), D, N.ptr(self.rows_dev), self.nobs,
                                               bw_ptr, N.ptr(self._lv_dev), N.ptr(self._tab), sh))
            tab = self._tab
        if out is not None:
            cands, datum, err = out
            if tuple(cands.shape) != (Nc, D) or datum.numel() < Nc or err.numel() < Nc:
                raise N.HbxError("sample: output tensors of the wrong size")
        else:
            cands = torch.empty((Nc, D), dtype=torch.float64, device=self.device)
            datum = torch.empty(Nc, dtype=torch.int64, device=self.device)
            err = torch.empty(Nc, dtype=torch.uint8, device=self.device)
        N.check(L.hbx_kde_sample(N.ptr(self.X_dev), D, N.ptr(self.rows_dev), self.nobs, bw_ptr,
                                 N.ptr(self._lv_dev), N.ptr(tab), float(bw_factor), int(seed) & (2 ** 64 - 1),
                                 int(counter_base) & (2 ** 64 - 1), int(stream_id) & 0xFFFFFFFF, Nc, N.ptr(cands),
                                 N.ptr(datum), N.ptr(err), sh))
        return cands, datum, err

    def logpdf(self, cands, rtol=1e-5, stream=None):
        """ln pdf per candidate within ``rtol * max(1, |ln p|)`` (the north-star contract), through
        ``hbx_kde_logpdf_rtol``: the fp32 matrix-core estimate wherever its rigorous per-candidate bound
        guarantees that, fp64 log space on the device for the rest (candidates whose fp32 expansion
        cancels large terms -- next to outlying observations, beyond D = 32 -- and exact-only KDEs), ln of
        the exact fp64 pdf for KDEs with negative categorical factors.  Returns float64 [Nc]."""
        torch = _torch()
        L = N.lib()
        C = np.ascontiguousarray(np.asarray(cands, dtype=np.float64).reshape(-1, self.k_vars))
        Nc = C.shape[0]
        if Nc == 0:
            return np.zeros(0)
        with N.on_device(self.device, stream):
            c_dev = torch.from_numpy(C).to(self.device)
            out = torch.empty(Nc, dtype=torch.float64, device=self.device)
            sb = int(L.hbx_kde_logpdf_rtol_scratch_bytes(Nc))
            scr = torch.empty(sb, dtype=torch.uint8, device=self.device)
            sh = N.stream_handle(stream, self.device)
            self._order(sh)
            N.check(L.hbx_kde_logpdf_rtol(N.ptr(c_dev), Nc, self.k_vars, N.ptr(self.params), N.ptr(self.table),
                                          N.ptr(self.X_dev), N.ptr(self.rows_dev), self.dc_pad, self.du_pad,
                                          self.variant, float(rtol), N.ptr(out), N.ptr(scr), sb, sh))
            return out.cpu().numpy()

    def _logpdf_exact(self, C, stream):
        """ln pdf at the rows of C: fp64 log space (hbx_kde_logpdf_exact: no underflow, ~1e-15) where
        the KDE's factors are positive, else ln of the exact fp64 pdf."""
        torch = _torch()
        L = N.lib()
        if not (self.has_neg or self.nan_all or self.nconst):
            with N.on_device(self.device, stream):
                p_dev = torch.from_numpy(np.ascontiguousarray(C)).to(self.device)
                o = torch.empty(C.shape[0], dtype=torch.float64, device=self.device)
                sh = N.stream_handle(stream, self.device)
                self._order(sh)
                N.check(L.hbx_kde_logpdf_exact(N.ptr(p_dev), C.shape[0], self.k_vars, N.ptr(self.params),
                                               N.ptr(self.X_dev), N.ptr(self.rows_dev), N.ptr(o), sh))
                return o.cpu().numpy()
        exact = np.atleast_1d(self.pdf(C, stream=stream))
        with np.errstate(divide="ignore", invalid="ignore"):
            return np.log(exact)

    def logpdf_est(self, cand_dev, stream=None):
        """fp32 log-domain estimate per candidate -> (lpos, lneg, err) numpy arrays."""
        torch = _torch()
        L = N.lib()
        Nc = int(cand_dev.shape[0])
        with N.on_device(self.device, stream):
            est = torch.empty((Nc, 4), dtype=torch.float32, device=self.device)
            sh = N.stream_handle(stream, self.device)
            self._order(sh)
            N.check(L.hbx_kde_logpdf(N.ptr(cand_dev), Nc, self.k_vars, N.ptr(self.params), N.ptr(self.table),
                                     self.dc_pad, self.du_pad, self.variant, N.ptr(est), sh))
            e = est.cpu().numpy()
        return e[:, 0], e[:, 1], e[:, 2]


_LEVELS = {}  # (device, level bytes) -> the level counts on the device (one upload per space and device)


def _levels_on_device(key, lv, device):
    t = _LEVELS.get((str(device), key))
    if t is None:
        t = _LEVELS[(str(device), key)] = _torch().from_numpy(lv.copy()).to(device)
    return t


_FAST_FNS = None


def _torch_fast_fns():
    """torch's raw current-device and current-stream accessors (None where this torch lacks them)."""
    global _FAST_FNS
    if _FAST_FNS is None:
        torch = _torch()
        _FAST_FNS = (getattr(torch._C, "_cuda_getDevice", None), getattr(torch._C, "_cuda_getCurrentRawStream", None))
    return _FAST_FNS


class KDEPair(object):
    """The (good, bad) KDE pair of one budget -- BOHB's ``kde_models[budget]`` entry.

    Immutable once built; BOHB replaces the whole entry on refit (bohb.py:248-251), so a
    concurrent ``get_config`` always sees a consistent snapshot.
    """

    def __init__(self, good, bad):
        self.good = good
        self.bad = bad
        if (good.dc_pad, good.du_pad) != (bad.dc_pad, bad.du_pad):
            raise N.HbxError("good/bad KDEs prepared for different kernel buckets")
        self.nmax = max(good.nobs, bad.nobs)
        # per-call constants of acquire(): the prepared KDEs' device pointers and variant codes, the
        # workspace size per candidate count, the result record's offset (host overhead of a
        # get_config at the reference's 64 candidates is of the order of the GPU work)
        self._kde_args = (good.params.data_ptr(), good.table.data_ptr(), good.X_dev.data_ptr(),
                          good.rows_dev.data_ptr(), good.variant, bad.params.data_ptr(), bad.table.data_ptr(),
                          bad.X_dev.data_ptr(), bad.rows_dev.data_ptr(), bad.variant, good.dc_pad, good.du_pad,
                          self.nmax)
        self._wsb = {}
        self._roff = None
        self._home = good._home if good._home == bad._home else None  # (None: each KDE checks for itself)
        # the synchronous fast path's constants (acquire: a call on the model's own device)
        dev = good.device
        self._dev_index = dev.index if dev.index is not None else _torch().cuda.current_device()
        self._cur_dev, self._raw_stream = _torch_fast_fns()
        L = N.lib()
        self._ws_cache = {}  # (thread, Nc) -> workspace of synchronous calls made without one
        # the fixed arguments bound once on the native side: the synchronous call converts 11 arguments
        # instead of 25 (hbx_kde_acquire_bound)
        self._bound = None
        self._bound_fn = L.hbx_kde_acquire_bound
        self._free_fn = L.hbx_kde_pair_free
        self._bound = L.hbx_kde_pair_bind(good.k_vars, *self._kde_args)
        if not self._bound:
            raise N.HbxError("hbx_kde_pair_bind: %s" % L.hbx_last_error().decode())

    def __del__(self):
        b, self._bound = getattr(self, "_bound", None), None
        if b:
            self._free_fn(b)

    def __getitem__(self, key):  # cg.kde_models[b]['good'] like the reference dict
        if key == "good":
            return self.good
        if key == "bad":
            return self.bad
        raise KeyError(key)

    def keys(self):
        return ["good", "bad"]

    def _order(self, sh):
        """Order stream ``sh`` after both KDEs' preparation (DeviceKDE._order) unless it is their stream."""
        if sh != self._home:
            self.good._order(sh)
            self.bad._order(sh)

    def result_offset(self):
        """Byte offset of the AcqResult record inside an acquisition workspace."""
        return int(N.lib().hbx_kde_result_ptr(4096)) - 4096

    def workspace_bytes(self, Nc):
        wsb = self._wsb.get(Nc)
        if wsb is None:
            wsb = self._wsb[Nc] = int(N.lib().hbx_kde_workspace_bytes(int(Nc), self.nmax))
        return wsb

    def acquire(self, cands, index_base=0, logs=False, stream=None, workspace=None, sync=True, events=None,
                ties="pinned"):
        """Select the first index minimising max(1e-8, g)/max(l, 1e-8) over the candidates.

        ``cands``: [Nc, D] float64 (numpy or a device tensor).  Returns AcqResult (index -1 when no
        candidate has a finite score: the reference then falls back to a random configuration).
        With ``logs`` the fp32 ln l(x), ln g(x) estimates are returned as well.
        With ``sync=False`` the result stays on the device: returns the result tensor view.

        ``ties``: 'pinned' (default) -- the GPU's exact re-score is the reference's float64 arithmetic on
        the pinned numpy 1.26.4 bit for bit, so its pick is final; 'process' -- candidates flagged
        ACQ_NEAR_TIE (within the spread another numpy build's exp could cause) are re-scored with this
        process's numpy (exact_host), reproducing what the reference would pick in this environment.
        """
        if ties not in ("pinned", "process"):
            raise ValueError("ties must be 'pinned' or 'process'")
        if (sync and not logs and stream is None and self._cur_dev is not None and self._raw_stream is not None
                and self._cur_dev() == self._dev_index):
            r = self._acquire_sync(cands, index_base, workspace, events)
            if r is not None:
                if ties == "process" and r.flags & ACQ_NEAR_TIE:
                    with N.on_device(self.good.device):
                        ws = workspace if workspace is not None else self._ws_cache[(threading.get_ident(), len(cands))]
                        self._resolve(r, ws, len(cands), len(cands), cands, int(index_base))
                return r
        with N.on_device(self.good.device, stream):
            return self._acquire(cands, index_base, logs, stream, workspace, sync, events, ties)

    def _acquire_sync(self, cands, index_base, workspace, events):
        """The drop-in's common call -- synchronous, the winner only, on the model's device and its current
        stream, which is this thread's current device (no device switch): one native call
        (hbx_kde_acquire_bound) with the fewest host steps around it; a workspace is kept per thread and
        candidate count when none is given.  None when the candidates need staging (host arrays, other
        dtypes): the general path then runs."""
        torch = _torch()
        if type(cands) is not torch.Tensor or cands.dtype is not torch.float64 or not cands.is_cuda:
            return None
        D = self.good.k_vars
        if cands.dim() != 2 or cands.shape[1] != D or not cands.is_contiguous() or \
                cands.device.index != self._dev_index:
            return None
        Nc = cands.shape[0]
        wsb = self._wsb.get(Nc)
        if wsb is None:
            wsb = self.workspace_bytes(Nc)
        if workspace is None:
            key = (threading.get_ident(), Nc)
            workspace = self._ws_cache.get(key)
            if workspace is None:
                workspace = self._ws_cache[key] = torch.empty(wsb, dtype=torch.uint8, device=cands.device)
        n = workspace.numel()
        if n < wsb:
            raise N.HbxError("workspace too small")
        rec = _record_buffer()
        sh = self._raw_stream(self._dev_index)
        if sh != self._home:
            self._order(sh)
        N.check(self._bound_fn(self._bound, cands.data_ptr(), Nc, int(index_base), workspace.data_ptr(), n, None,
                               events.address if events is not None else None, sh, rec, None))
        return AcqResult.from_bytes(rec.raw[:RESULT_BYTES])

    def _acquire(self, cands, index_base, logs, stream, workspace, sync, events, ties):
        torch = _torch()
        L = N.lib()
        dev = self.good.device
        if isinstance(cands, np.ndarray):
            c_dev = torch.from_numpy(np.ascontiguousarray(cands, dtype=np.float64)).to(dev)
        else:
            c_dev = cands
            if c_dev.dtype != torch.float64 or not c_dev.is_contiguous():
                raise N.HbxError("candidate tensor must be contiguous float64 [Nc, D]")
        Nc = int(c_dev.shape[0])
        D = self.good.k_vars
        if Nc > 0 and (c_dev.dim() != 2 or int(c_dev.shape[1]) != D):
            raise N.HbxError("candidates must be [Nc, %d], got %s" % (D, tuple(c_dev.shape)))
        wsb = self.workspace_bytes(Nc)
        ws = workspace if workspace is not None else torch.empty(wsb, dtype=torch.uint8, device=dev)
        if ws.numel() < wsb:
            raise N.HbxError("workspace too small")
        logl = torch.empty(Nc, dtype=torch.float32, device=dev) if logs else None
        logg = torch.empty(Nc, dtype=torch.float32, device=dev) if logs else None
        wsp = ws.data_ptr()
        sh = N.stream_handle(stream, dev)
        self._order(sh)
        if sync and not logs:  # one native call: the acquisition and its record on the host
            rec = _record_buffer()
            N.check(self._bound_fn(self._bound, c_dev.data_ptr(), Nc, int(index_base), wsp, ws.numel(), None,
                                   events.address if events is not None else None, sh, rec, None))
            res = AcqResult.from_bytes(rec.raw[:RESULT_BYTES])
            if ties == "process" and res.flags & ACQ_NEAR_TIE:
                self._resolve(res, ws, Nc, Nc, cands if isinstance(cands, np.ndarray) else c_dev, int(index_base))
            return res
        N.check(L.hbx_kde_acquire(c_dev.data_ptr(), Nc, D, int(index_base), *self._kde_args,
                                  N.ptr(logl), N.ptr(logg), wsp, ws.numel(),
                                  events.address if events is not None else None, sh))
        if self._roff is None:
            self._roff = int(L.hbx_kde_result_ptr(wsp)) - wsp
        off = self._roff
        rview = ws[off:off + RESULT_BYTES]
        if not sync:
            return rview
        res = AcqResult.from_bytes(fetch_bytes(rview, stream))
        if ties == "process" and res.flags & ACQ_NEAR_TIE:
            self._resolve(res, ws, Nc, Nc, cands if isinstance(cands, np.ndarray) else c_dev, int(index_base))
        if logs:
            return res, logl.cpu().numpy(), logg.cpu().numpy()
        return res

    def _ws_offsets(self, Nc, seg):
        o = np.zeros(5, dtype=np.int64)
        N.check(N.lib().hbx_kde_ws_offsets(int(Nc), int(max(seg, 1)), self.nmax, N.ptr(o)))
        return [int(v) for v in o]

    def _resolve(self, res, ws, Nc, seg, cands, index_base):
        """HBX_ACQ_NEAR_TIE on a single acquisition: re-score the near set in the reference's numpy
        arithmetic and take its strict-'<' first-index minimum (exact_host.resolve)."""
        from . import exact_host
        o = self._ws_offsets(Nc, seg)
        idx = ws[o[2]:o[2] + 4 * res.near].view(_torch().int32).cpu().numpy().astype(np.int64)
        pick = exact_host.resolve(self.good, self.bad, _rows_of(cands, idx), idx)
        if pick is not None:
            res.index, res.score, res.pdf_l, res.pdf_g = pick[0] + index_base, pick[1], pick[2], pick[3]
        res.flags |= ACQ_RESOLVED

    def _resolve_batch(self, recs, ws, Nc, seg, cands):
        """HBX_ACQ_NEAR_TIE in a batched acquisition: the same, per flagged segment."""
        from . import exact_host
        torch = _torch()
        o = self._ws_offsets(Nc, seg)
        cnt = int(ws[o[0]:o[0] + 4].view(torch.int32).item())
        lst = ws[o[1]:o[1] + 4 * cnt].view(torch.int32).cpu().numpy().astype(np.int64)
        flg = ws[o[2]:o[2] + 4 * cnt].view(torch.int32).cpu().numpy()
        for b, r in enumerate(recs):
            if not r.flags & ACQ_NEAR_TIE:
                continue
            idx = np.sort(lst[(flg != 0) & (lst // seg == b)])
            pick = exact_host.resolve(self.good, self.bad, _rows_of(cands, idx), idx)
            if pick is not None:
                r.index, r.score, r.pdf_l, r.pdf_g = pick[0] - b * seg, pick[1], pick[2], pick[3]
            r.flags |= ACQ_RESOLVED

    def acquire_mapped(self, cands):
        """acquire(cands) for a host array from mapped_candidates(): the kernels read the candidates in host
        memory (zero copy), the pick comes back in the same synchronous call (hbx_kde_acquire_bound).  Falls
        back to acquire() off the fast path's conditions (another current device)."""
        if self._cur_dev is None or self._raw_stream is None or self._cur_dev() != self._dev_index:
            return self.acquire(np.array(cands))
        torch = _torch()
        Nc = cands.shape[0]
        wsb = self._wsb.get(Nc)
        if wsb is None:
            wsb = self.workspace_bytes(Nc)
        key = (threading.get_ident(), Nc)
        workspace = self._ws_cache.get(key)
        if workspace is None:
            workspace = self._ws_cache[key] = torch.empty(wsb, dtype=torch.uint8, device=self.good.device)
        rec = _record_buffer()
        sh = self._raw_stream(self._dev_index)
        if sh != self._home:
            self._order(sh)
        N.check(self._bound_fn(self._bound, cands.ctypes.data, Nc, 0, workspace.data_ptr(), workspace.numel(), None,
                               None, sh, rec, None))
        return AcqResult.from_bytes(rec.raw[:RESULT_BYTES])

    def acquire_pick(self, cands, err, workspace, row, sh=None):
        """One synchronous acquisition of ``cands`` (a device [Nc, D] f64 tensor on the model's device) with its
        whole pick on the host after ONE wait (hbx_kde_acquire_bound with err and row_out): the record, whether
        any ``err`` flag (the GPU sampler's per-candidate domain errors, a device u8 tensor or None) is set
        (ACQ_DOMAIN_ERR in ``flags``), and the winning row written into ``row`` (a host f64 array of D).
        ``sh``: the stream handle (default: the device's current stream).  Returns the AcqResult."""
        if sh is None:
            sh = N.stream_handle(None, self.good.device)
        if sh != self._home:
            self._order(sh)
        rec = _record_buffer()
        N.check(self._bound_fn(self._bound, cands.data_ptr(), int(cands.shape[0]), 0, workspace.data_ptr(),
                               workspace.numel(), err.data_ptr() if err is not None else None, None, sh, rec,
                               row.ctypes.data))
        return AcqResult.from_bytes(rec.raw[:RESULT_BYTES])

    def batch_workspace_bytes(self, Nc, seg):
        return int(N.lib().hbx_kde_batch_workspace_bytes(int(Nc), int(seg), self.nmax))

    def acquire_batch(self, cands, seg, stream=None, workspace=None, results=None, sync=True, ties="pinned"):
        """B = ceil(Nc/seg) acquisitions in one pass: candidates [b*seg, (b+1)*seg) are the candidates
        of get_config call b.  Returns a list of B AcqResult (index relative to the segment start).
        With ``sync=False`` returns the device tensor of the B raw records instead."""
        if ties not in ("pinned", "process"):
            raise ValueError("ties must be 'pinned' or 'process'")
        with N.on_device(self.good.device, stream):
            return self._acquire_batch(cands, seg, stream, workspace, results, sync, ties)

    def _acquire_batch(self, cands, seg, stream, workspace, results, sync, ties):
        torch = _torch()
        L = N.lib()
        dev = self.good.device
        if isinstance(cands, np.ndarray):
            c_dev = torch.from_numpy(np.ascontiguousarray(cands, dtype=np.float64)).to(dev)
        else:
            c_dev = cands
            if c_dev.dtype != torch.float64 or not c_dev.is_contiguous():
                raise N.HbxError("candidate tensor must be contiguous float64 [Nc, D]")
        Nc, seg = int(c_dev.shape[0]), int(seg)
        D = self.good.k_vars
        if seg < 1:
            raise N.HbxError("segment length must be >= 1")
        if Nc > 0 and (c_dev.dim() != 2 or int(c_dev.shape[1]) != D):
            raise N.HbxError("candidates must be [Nc, %d], got %s" % (D, tuple(c_dev.shape)))
        B = (Nc + seg - 1) // seg
        wsb = self.batch_workspace_bytes(Nc, seg)
        ws = workspace if workspace is not None else torch.empty(wsb, dtype=torch.uint8, device=dev)
        if ws.numel() < wsb:
            raise N.HbxError("workspace too small")
        out = results if results is not None else torch.empty(max(B, 1) * RESULT_BYTES, dtype=torch.uint8, device=dev)
        if out.numel() < B * RESULT_BYTES:
            raise N.HbxError("result buffer too small")
        g, b = self.good, self.bad
        sh = N.stream_handle(stream, dev)
        self._order(sh)
        N.check(L.hbx_kde_acquire_batch(N.ptr(c_dev), Nc, seg, D, 0,
                                        N.ptr(g.params), N.ptr(g.table), N.ptr(g.X_dev), N.ptr(g.rows_dev), g.variant,
                                        N.ptr(b.params), N.ptr(b.table), N.ptr(b.X_dev), N.ptr(b.rows_dev), b.variant,
                                        g.dc_pad, g.du_pad, self.nmax, None, None, N.ptr(out), N.ptr(ws), ws.numel(),
                                        sh))
        if not sync:
            return out[:B * RESULT_BYTES]
        raw = fetch_bytes(out[:B * RESULT_BYTES], stream)
        recs = [AcqResult.from_bytes(raw[i * RESULT_BYTES:(i + 1) * RESULT_BYTES]) for i in range(B)]
        if ties == "process" and any(r.flags & ACQ_NEAR_TIE for r in recs):
            self._resolve_batch(recs, ws, Nc, seg, cands if isinstance(cands, np.ndarray) else c_dev)
        return recs


class ScoreEvents(object):
    """Three hipEvents bracketing the two scoring launches of one acquisition (bench timing)."""

    def __init__(self):
        import ctypes
        L = N.lib()
        self._ev = (ctypes.c_void_p * 3)()
        for i in range(3):
            h = ctypes.c_void_p()
            N.check(L.hbx_event_create(ctypes.addressof(h)))
            self._ev[i] = h.value
        self.address = ctypes.addressof(self._ev)

    def elapsed_ms(self, fused=False):
        """(l launch ms, g launch ms) of the last recorded acquisition (events must be complete).
        ``fused``: l and g ran as one pair launch, which records only events 0 and 1 -> (l+g, 0)."""
        import ctypes
        L = N.lib()
        a, b = ctypes.c_float(), ctypes.c_float()
        N.check(L.hbx_event_elapsed_ms(self._ev[0], self._ev[1], ctypes.addressof(a)))
        if fused:
            return a.value, 0.0
        N.check(L.hbx_event_elapsed_ms(self._ev[1], self._ev[2], ctypes.addressof(b)))
        return a.value, b.value

    def __del__(self):
        try:
            L = N.lib()
            for i in range(3):
                L.hbx_event_destroy(self._ev[i])
        except Exception:
            pass


def split_sizes(n, D, min_points, top_n_percent=15, split_rule="bohb"):
    """(n_good, n_bad) clipped to n, or None where the reference returns without building a model.

    'bohb': integer floor sizes (bohb.py:224-225), a model needs rows > D (bohb.py:234-237);
    'kde_ei': int(max(top% * N / 100., mp)) (kde_ei.py:190-191), rows >= D (rows == D raises in
    KDEMultivariate, kernel_density.py:107-109, as in the reference).
    """
    if split_rule == "bohb":
        n_good, n_bad = bohb_split_sizes(n, min_points, top_n_percent)
        if min(n_good, n) <= D or min(n_bad, n) <= D:
            return None
    else:
        n_good = int(max(top_n_percent * n / 100., min_points))
        n_bad = int(max((100 - top_n_percent) * n / 100., min_points))
        if min(n_good, n) < D or min(n_bad, n) < D:
            return None
        if min(n_good, n) <= D or min(n_bad, n) <= D:
            raise ValueError("The number of observations must be larger than the number of variables.")
    # numpy slicing semantics: idx[:n_good] / idx[-n_bad:] clip at n
    return min(n_good, n), min(n_bad, n)


class _DevSlice(object):
    """A piece of a device allocation by address (a refit's parameter blocks and tables): what the engine
    reads of them is the address (``data_ptr``) and the size (``numel``); ``base`` keeps the allocation."""
    __slots__ = ("base", "_ptr", "_numel")

    def __init__(self, base, ptr, numel):
        self.base, self._ptr, self._numel = base, ptr, numel

    def data_ptr(self):
        return self._ptr

    def numel(self):
        return self._numel


def _raw_stream(device):
    """The device's current HIP stream handle (torch's raw accessor where it exists)."""
    torch = _torch()
    f = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    if f is not None:
        return f(device.index if device.index is not None else torch.cuda.current_device())
    return torch.cuda.current_stream(device).cuda_stream


class ObservationStore(object):
    """One budget's observations (``get_array()`` rows and losses) resident in HBM, appended to as
    results arrive (bohb.py:211-213), so a refit moves only the new rows to the device: one pinned
    host->device copy, one ``hbx_kde_refit`` call (split, bandwidths, level counts, both KDEs'
    preparation; no host synchronisation inside) and one device->host copy of the split and bandwidths.

    Each refit returns a new immutable KDEPair; rows already on the device are never rewritten, so
    models handed out earlier stay valid while later rows are appended (growth reallocates).
    """

    def __init__(self, D, var_type, device=None, capacity=256):
        self.D = int(D)
        self.var_type = var_type
        self.vt = np.ascontiguousarray(var_type_codes(var_type))
        self.device = device or default_device()
        self.n = 0          # rows on the device
        self.nh = 0         # rows on the host (added)
        self._hcap = 0
        self._Xh = self._lh = None
        self._cap = 0
        self.X_dev = self.loss_dev = None
        self._init_cap = int(capacity)
        self.dc_pad, self.du_pad = scoring_bucket(self.vt)

    def _reserve(self, n):
        torch = _torch()
        if n <= self._cap:
            return
        cap = max(self._init_cap, self._cap)
        while cap < n:
            cap *= 2
        X = torch.empty((cap, self.D), dtype=torch.float64, device=self.device)
        L = torch.empty(cap, dtype=torch.float64, device=self.device)
        if self.n:
            X[:self.n].copy_(self.X_dev[:self.n])
            L[:self.n].copy_(self.loss_dev[:self.n])
        self.X_dev, self.loss_dev, self._cap = X, L, cap

    def add(self, rows, losses):
        """Append observations on the host side (O(rows x D)); the next refit moves them."""
        rows = np.asarray(rows, dtype=np.float64).reshape(-1, self.D)
        losses = np.asarray(losses, dtype=np.float64).reshape(-1)
        if losses.shape[0] != rows.shape[0]:
            raise N.HbxError("observation store: %d rows, %d losses" % (rows.shape[0], losses.shape[0]))
        cat = self.vt != 0
        if cat.any():  # checked before the rows enter the store: a bad row would fail every later refit
            codes = rows[:, cat]
            if not (np.all((codes >= 0) & (codes < 1024)) and np.all(codes == np.floor(codes))):
                raise N.HbxError("categorical codes must be integers in [0, 1024)")
        m = self.nh + rows.shape[0]
        if m > self._hcap:
            cap = max(self._init_cap, self._hcap)
            while cap < m:
                cap *= 2
            Xh = np.empty((cap, self.D))
            lh = np.empty(cap)
            if self.nh:
                Xh[:self.nh] = self._Xh[:self.nh]
                lh[:self.nh] = self._lh[:self.nh]
            self._Xh, self._lh, self._hcap = Xh, lh, cap
        self._Xh[self.nh:m] = rows
        self._lh[self.nh:m] = losses
        self.nh = m

    @property
    def X_host(self):
        return self._Xh[:self.nh]

    @property
    def losses_host(self):
        return self._lh[:self.nh]

    def refit(self, min_points, top_n_percent=15, split_rule="bohb", stream=None):
        """Refit on every row added so far (bohb.py:220-251).  Returns a KDEPair, or None where the reference
        builds no model (too few rows for a KDE, bohb.py:234-237).  The row-count gate before it
        (``len <= min_points + 1``: no refit, bohb.py:216-217) is the caller's, as in new_result."""
        n = self.nh
        sizes = split_sizes(n, self.D, min_points, top_n_percent, split_rule)
        if sizes is None:
            return None
        cur, _ = _torch_fast_fns()
        if stream is None and cur is not None and self.device.index is not None and cur() == self.device.index:
            return self._refit(self._Xh[:n], self._lh[:n], n, sizes, stream)  # (already current: no context)
        with N.on_device(self.device, stream):
            return self._refit(self._Xh[:n], self._lh[:n], n, sizes, stream)

    def _refit(self, X_host, losses, n, sizes, stream):
        torch = _torch()
        L = N.lib()
        D = self.D
        n_good, n_bad = sizes
        n_new = n - self.n
        self._reserve(n)
        sh = stream.cuda_stream if stream is not None else _raw_stream(self.device)
        # the new rows then their losses, from host memory: the native call carries up to 256 doubles in the
        # refit launch's arguments (no copy), more through its scratch
        staged = None
        if n_new:
            staged = np.empty(n_new * (D + 1), dtype=np.float64)
            staged[:n_new * D] = X_host[self.n:].reshape(-1)
            staged[n_new * D:] = losses[self.n:]
        # every device block of the refit in ONE allocation (views: out, scratch, parameter blocks, tables)
        ob = int(L.hbx_kde_refit_out_bytes(n, D))
        sb = int(L.hbx_kde_refit_scratch_bytes(n, D))
        pb = int(L.hbx_kde_param_bytes())
        tgf = int(L.hbx_kde_table_floats(n_good, self.dc_pad, self.du_pad))
        tbf = int(L.hbx_kde_table_floats(n_bad, self.dc_pad, self.du_pad))
        a_ob, a_sb, a_pb, a_tg = (ob + 255) & ~255, (sb + 255) & ~255, (pb + 255) & ~255, (4 * tgf + 255) & ~255
        blk = torch.empty(a_ob + a_sb + 2 * a_pb + a_tg + 4 * tbf, dtype=torch.uint8, device=self.device)
        # 256-byte aligned pieces: out | scratch | params good | params bad | table good | table bad
        p0 = blk.data_ptr()
        p_scr = p0 + a_ob
        pg = _DevSlice(blk, p_scr + a_sb, pb)
        pbad = _DevSlice(blk, pg._ptr + a_pb, pb)
        tg = _DevSlice(blk, pbad._ptr + a_pb, tgf)
        tb = _DevSlice(blk, tg._ptr + a_tg, tbf)
        # the output block lands in a fresh host array when the call returns (published by the preparation's
        # last workgroups through mapped host memory): its pieces are views, no copies
        ah = np.empty(ob, dtype=np.uint8)
        N.check(L.hbx_kde_refit_sync(N.ptr(self.X_dev), N.ptr(self.loss_dev), n, D, N.ptr(self.vt),
                                     staged.ctypes.data if staged is not None else None, n_new, n_good, n_bad,
                                     bandwidth_factor(n_good, D), bandwidth_factor(n_bad, D), pg._ptr,
                                     tg._ptr, tgf, pbad._ptr, tb._ptr, tbf, p0, p_scr, sb, sh, ah.ctypes.data))
        order_h = ah[:8 * n].view(np.int64)
        o = 8 * n
        bw_gh = ah[o:o + 8 * D].view(np.float64)
        bw_bh = ah[o + 8 * D:o + 16 * D].view(np.float64)
        nl_gh = ah[o + 16 * D:o + 20 * D].view(np.int32)
        nl_bh = ah[o + 20 * D:o + 24 * D].view(np.int32)
        info_g = ah[o + 24 * D:o + 24 * D + 32].view(np.int32)
        info_b = ah[o + 24 * D + 32:o + 24 * D + 64].view(np.int32)  # (level counts < 0: the call failed)
        self.n = n  # the rows count as resident only once the refit has completed and validated
        order = blk[:8 * n].view(torch.int64)
        X_dev = self.X_dev
        good = DeviceKDE(X_dev, order[:n_good], self.var_type, bw_gh, nl_gh, (X_host, order_h[:n_good]),
                         prepared=(pg, tg, info_g), home=sh)
        bad = DeviceKDE(X_dev, order[n - n_bad:], self.var_type, bw_bh, nl_bh, (X_host, order_h[n - n_bad:]),
                        prepared=(pbad, tb, info_b), home=sh)
        pair = KDEPair(good, bad)
        pair._keep = (blk,)  # the rows tensors are views of the refit's block
        return pair


def fit_pair(configs, losses, var_type, min_points, top_n_percent=15, device=None, stream=None,
             split_rule="bohb"):
    """Refit the good/bad KDEs of one budget on the GPU (BOHB.new_result, bohb.py:220-251) from host
    arrays: all rows staged at once through an ObservationStore.

    Returns a KDEPair, or None where the reference returns without building a model.
    ``split_rule`` 'bohb' uses integer floor sizes (bohb.py:224-225) and requires rows > D;
    'kde_ei' uses int(max(top%*N/100., mp)) (kde_ei.py:190-191) and requires rows >= D.
    """
    X = np.ascontiguousarray(np.asarray(configs, dtype=np.float64))
    n, D = X.shape
    store = ObservationStore(D, var_type, device=device, capacity=max(n, 1))
    store.add(X, losses)
    return store.refit(min_points, top_n_percent, split_rule, stream=stream)


def fit_pair_from_rows(X, good_rows, bad_rows, var_type, bw_good, bw_bad, nlev_good, nlev_bad, device=None):
    """Build a KDEPair from an explicit split and bandwidths (tests / externally fitted models)."""
    torch = _torch()
    device = device or default_device()
    X = np.ascontiguousarray(np.asarray(X, dtype=np.float64))
    with N.on_device(device):
        X_dev = torch.from_numpy(X).to(device)
        rg = torch.from_numpy(np.asarray(good_rows, dtype=np.int64)).to(device)
        rb = torch.from_numpy(np.asarray(bad_rows, dtype=np.int64)).to(device)
        good = DeviceKDE(X_dev, rg, var_type, bw_good, nlev_good, X[np.asarray(good_rows)])
        bad = DeviceKDE(X_dev, rb, var_type, bw_bad, nlev_bad, X[np.asarray(bad_rows)])
    return KDEPair(good, bad)
