"""ctypes binding of libhbx.so (include/hbx.h).

The engine has exactly one compute path: the HIP kernels in this library.  There is no CPU
fallback -- if the library is missing or cannot be loaded, every engine call raises.
"""

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# HBX_LIB_PATH: load another build of the same library (diagnostic ablation builds, tools/ablate.sh)
LIB_PATH = os.environ.get("HBX_LIB_PATH") or os.path.join(_HERE, "_lib", "libhbx.so")
DIAGNOSTIC_BUILD = bool(os.environ.get("HBX_LIB_PATH"))

_lock = threading.Lock()
_lib = None

c_i32, c_i64, c_f64p, c_vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p

# name -> (restype, argtypes); every pointer is passed as an integer address (c_void_p)
SIGNATURES = {
    "hbx_last_error": (ctypes.c_char_p, []),
    "hbx_version": (ctypes.c_char_p, []),
    "hbx_kde_param_bytes": (c_i64, []),
    "hbx_kde_param_bw_offset": (c_i64, []),
    "hbx_kde_est_bytes": (c_i64, []),
    "hbx_acq_result_bytes": (c_i64, []),
    "hbx_max_dims": (c_i32, []),
    "hbx_sort_scratch_bytes": (c_i64, [c_i64]),
    "hbx_seg_argsort": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "hbx_kde_fit": (c_i32, [c_vp, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                            c_vp, c_vp]),
    "hbx_kde_bucket": (c_i32, [c_i32, c_i32, c_vp, c_vp, c_vp]),
    "hbx_kde_table_floats": (c_i64, [c_i32, c_i32, c_i32]),
    "hbx_kde_prepare": (c_i32, [c_vp, c_i32, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "hbx_kde_refit_out_bytes": (c_i64, [c_i64, c_i32]),
    "hbx_kde_refit_scratch_bytes": (c_i64, [c_i64, c_i32]),
    "hbx_kde_refit": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_i64, c_i64, c_i64, ctypes.c_double,
                              ctypes.c_double, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "hbx_kde_refit_sync": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_i64, c_i64, c_i64, ctypes.c_double,
                                   ctypes.c_double, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64,
                                   c_vp, c_vp]),
    "hbx_stream_order": (c_i32, [c_vp, c_vp]),
    "hbx_kde_logpdf": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp]),
    "hbx_kde_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "hbx_kde_acquire": (c_i32, [c_vp, c_i64, c_i32, c_i64,
                                c_vp, c_vp, c_vp, c_vp, c_i32,
                                c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32,
                                c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "hbx_kde_pair_bind": (c_vp, [c_i32, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32,
                                 c_i64]),
    "hbx_kde_acquire_bound": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "hbx_kde_pair_free": (None, [c_vp]),
    "hbx_kde_batch_workspace_bytes": (c_i64, [c_i64, c_i64, c_i64]),
    "hbx_kde_acquire_batch": (c_i32, [c_vp, c_i64, c_i64, c_i32, c_i64,
                                      c_vp, c_vp, c_vp, c_vp, c_i32,
                                      c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32,
                                      c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "hbx_philox4x32_10": (c_i32, [c_vp, c_vp, c_vp]),
    "hbx_kde_sample": (c_i32, [c_vp, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, ctypes.c_double, ctypes.c_uint64,
                               ctypes.c_uint64, ctypes.c_uint32, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "hbx_norm_ppf": (c_i32, [c_vp, c_i64, c_vp, c_vp]),
    "hbx_kde_sample_table_bytes": (c_i64, [c_i64, c_i32]),
    "hbx_kde_sample_table": (c_i32, [c_vp, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "hbx_kde_cv_terms": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_double,
                                 ctypes.c_double, ctypes.c_double, c_vp, c_vp, c_vp]),
    "hbx_event_create": (c_i32, [c_vp]),
    "hbx_event_destroy": (c_i32, [c_vp]),
    "hbx_event_elapsed_ms": (c_i32, [c_vp, c_vp, c_vp]),
    "hbx_kde_result_ptr": (c_vp, [c_vp]),
    "hbx_fetch": (c_i32, [c_vp, c_vp, c_i64, c_vp]),
    "hbx_mapped_host_buffers": (c_i64, []),
    "hbx_kde_ws_offsets": (c_i32, [c_i64, c_i64, c_i64, c_vp]),
    "hbx_np_exp": (c_i32, [c_vp, c_i64, c_vp, c_vp]),
    "hbx_kde_pdf_scratch_bytes": (c_i64, [c_i64]),
    "hbx_kde_pdf_exact": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "hbx_kde_logpdf_exact": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "hbx_rccl_unique_id_bytes": (c_i64, []),
    "hbx_rccl_get_unique_id": (c_i32, [c_vp]),
    "hbx_rccl_comm_init": (c_i32, [c_vp, c_i32, c_vp, c_i32, c_i32]),
    "hbx_rccl_comm_count": (c_i32, [c_vp, c_vp]),
    "hbx_rccl_comm_destroy": (c_i32, [c_vp]),
    "hbx_argmax_gather_bytes": (c_i64, [c_i32]),
    "hbx_argmax_allreduce": (c_i32, [c_vp, c_vp, c_vp, c_i32, c_vp, c_vp]),
    "hbx_argmax_records": (c_i32, [c_vp, c_i32, c_vp, c_vp]),
    "hbx_sh_promote": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "hbx_seg_argsort_ex": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_i32, c_vp]),
    "hbx_sh_promote_scratch_bytes": (c_i64, [c_i64, c_i64, c_i64, c_i32, c_i32]),
    "hbx_sh_promote_ex": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32,
                                  c_vp, c_vp]),
    "hbx_sh_promote_one": (c_i32, [c_vp, c_i64, ctypes.c_double, c_vp, c_vp, c_i32, c_vp, c_i32, c_vp]),
    "hbx_sh_advance_mapped": (c_i32, [c_vp, c_i64, ctypes.c_double, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_i32,
                                      c_vp]),
    "hbx_sh_advance_state": (c_i32, [c_vp, c_i64, ctypes.c_double, c_vp]),
    "hbx_host_alloc": (c_i32, [c_i64, c_vp]),
    "hbx_kde_logpdf_rtol_scratch_bytes": (c_i64, [c_i64]),
    "hbx_kde_logpdf_rtol": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, ctypes.c_double,
                                    c_vp, c_vp, c_i64, c_vp]),
    "hbx_host_free": (c_i32, [c_vp]),
    "hbx_np_argsort_host": (c_i32, [c_vp, c_i64, c_vp]),
    "hbx_sh_advance_host": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_vp]),
    "hbx_mt_state_bytes": (c_i64, []),
    "hbx_mt_draw": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_vp]),
    "hbx_bohb_draw": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, ctypes.c_double, c_i64, c_vp, c_vp, c_vp, c_vp,
                              c_vp, c_vp, c_vp]),
}

# tie order of the sorts (include/hbx.h): numpy's unstable argsort (the reference's) or by position
ORDER_NUMPY = 0
ORDER_STABLE = 1


def order_mode(name):
    """'numpy' (the reference's tie order, default) or 'stable' -> the HBX_ORDER_* code."""
    if name in ("numpy", ORDER_NUMPY):
        return ORDER_NUMPY
    if name in ("stable", ORDER_STABLE):
        return ORDER_STABLE
    raise ValueError("tie order must be 'numpy' or 'stable', got %r" % (name,))


class HbxError(RuntimeError):
    pass


def lib():
    """Load libhbx.so (once).  Raises if it is not built: there is no fallback path."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise HbxError("libhbx.so not found at %s -- build it with `python -m hpbandster_amd.build` "
                           "(the engine has no CPU fallback)" % LIB_PATH)
        # torch first: its bundled libamdhip64.so.7 then satisfies libhbx's HIP dependency (same
        # SONAME), so kernels and torch's allocator/streams share one HIP runtime.
        import torch  # noqa: F401
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if DIAGNOSTIC_BUILD and not hasattr(L, name):  # an older build under A/B: entries it lacks stay absent
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
        return _lib


def check(rc):
    if rc != 0:
        msg = lib().hbx_last_error()
        raise HbxError("libhbx error %d: %s" % (rc, msg.decode() if msg else "?"))


def call(name, *args):
    check(getattr(lib(), name)(*args))


def ptr(t):
    """Device/host address of a torch tensor or numpy array (None -> NULL)."""
    if t is None:
        return None
    if hasattr(t, "data_ptr"):
        return t.data_ptr()
    return t.ctypes.data


def stream_handle(stream=None, device=None):
    """hipStream_t of ``stream``, else torch's current stream of ``device`` (not of the calling thread's
    current device: a dispatcher thread's current device is 0 whatever device the model lives on)."""
    import torch
    if stream is not None:
        return stream.cuda_stream
    raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    if raw is not None:  # the raw handle, without building a Stream object per engine call
        idx = None if device is None else device if isinstance(device, int) else torch.device(device).index
        return raw(torch.cuda.current_device() if idx is None else int(idx))
    return torch.cuda.current_stream(device).cuda_stream


class on_device(object):
    """Context of one engine call: ``device`` current (so torch's copies and allocations land there) and,
    with an explicit ``stream``, that stream current too -- the host<->device copies torch enqueues and
    the kernels libhbx enqueues are then ordered on one stream."""

    def __init__(self, device, stream=None):
        import torch
        self._ctx = [torch.cuda.device(device)]
        if stream is not None:
            self._ctx.append(torch.cuda.stream(stream))

    def __enter__(self):
        for c in self._ctx:
            c.__enter__()
        return self

    def __exit__(self, *exc):
        for c in reversed(self._ctx):
            c.__exit__(*exc)
        return False
