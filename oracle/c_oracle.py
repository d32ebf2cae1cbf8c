"""ORACLE -- test infrastructure only: ctypes wrapper of oracle/_build/libkde_oracle.so."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_build", "libkde_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            build()
        L = ctypes.CDLL(SO)
        vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
        L.oracle_kde_pdf.argtypes = [vp, i64, i32, vp, vp, vp, vp, i64, vp, i32]
        L.oracle_kde_pdf.restype = None
        L.oracle_kde_pdf_mode.argtypes = [vp, i64, i32, vp, vp, vp, vp, i64, vp, i32, i32]
        L.oracle_kde_pdf_mode.restype = None
        L.oracle_np_exp.argtypes = [vp, i64, vp]
        L.oracle_np_exp.restype = None
        L.oracle_bohb_select.argtypes = [vp, vp, i64, vp]
        L.oracle_bohb_select.restype = i64
        L.oracle_max_threads.restype = i32
        L.oracle_kde_pdf_screen.argtypes = [vp, i64, i32, vp, vp, vp, vp, i64, vp, vp, i32]
        L.oracle_kde_pdf_screen.restype = i32
        _lib = L
    return _lib


def np_exp(x):
    """numpy 1.26.4's float64 exp (the pinned reference's), bit for bit (oracle/np_arith.h)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    lib().oracle_np_exp(x.ctypes.data, x.size, y.ctypes.data)
    return y


def kde_pdf(data, bw, var_type, nlev, pts, nthreads=0, exact=False):
    """KDEMultivariate.pdf at pts.  exact=True: the reference's float64 arithmetic bit for bit
    (numpy 1.26.4's exp and pairwise sums); False: libm exp, sequential sums (CPU baseline)."""
    data = np.ascontiguousarray(data, dtype=np.float64)
    pts = np.ascontiguousarray(np.atleast_2d(pts), dtype=np.float64)
    vt = np.array([0 if c == "c" else 1 for c in var_type], dtype=np.int32)
    bw = np.ascontiguousarray(bw, dtype=np.float64)
    nlev = np.ascontiguousarray(nlev, dtype=np.int32)
    out = np.empty(pts.shape[0])
    lib().oracle_kde_pdf_mode(data.ctypes.data, data.shape[0], data.shape[1], vt.ctypes.data, bw.ctypes.data,
                              nlev.ctypes.data, pts.ctypes.data, pts.shape[0], out.ctypes.data, int(nthreads),
                              1 if exact else 0)
    return out


def kde_pdf_screen(data, bw, var_type, nlev, pts, nthreads=0):
    """Screening pdf (one libm exp per pair, kde_oracle.c:oracle_kde_pdf_screen) and its per-point
    relative bound against the exact mode; None when a categorical kernel is not positive."""
    data = np.ascontiguousarray(data, dtype=np.float64)
    pts = np.ascontiguousarray(np.atleast_2d(pts), dtype=np.float64)
    vt = np.array([0 if c == "c" else 1 for c in var_type], dtype=np.int32)
    bw = np.ascontiguousarray(bw, dtype=np.float64)
    nlev = np.ascontiguousarray(nlev, dtype=np.int32)
    out = np.empty(pts.shape[0])
    rel = np.empty(pts.shape[0])
    rc = lib().oracle_kde_pdf_screen(data.ctypes.data, data.shape[0], data.shape[1], vt.ctypes.data, bw.ctypes.data,
                                     nlev.ctypes.data, pts.ctypes.data, pts.shape[0], out.ctypes.data,
                                     rel.ctypes.data, int(nthreads))
    if rc != 0:
        return None
    return out, rel


def bohb_select(pdf_l, pdf_g):
    l = np.ascontiguousarray(pdf_l, dtype=np.float64)
    g = np.ascontiguousarray(pdf_g, dtype=np.float64)
    best = np.zeros(1)
    i = lib().oracle_bohb_select(l.ctypes.data, g.ctypes.data, l.shape[0], best.ctypes.data)
    return int(i), float(best[0])
