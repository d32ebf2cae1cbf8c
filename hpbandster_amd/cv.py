"""Cross-validated KDE bandwidths on the GPU: KDEMultivariate(bw='cv_ls' | 'cv_ml').

The reference's KernelDensityEstimator generator fits its model with
``sm.nonparametric.KDEMultivariate(data, var_type, bw='cv_ls')`` (kde.py:145-147).  statsmodels 0.12.2
selects that bandwidth with ``scipy.optimize.fmin`` (Nelder-Mead) from the normal-reference rule
(SM:_kernel_base.py:279-332), evaluating an O(n^2 D) objective at every simplex step:

* ``imse(bw)`` (cv_ls, SM:kernel_density.py:246-332): F / n^2 - 2 L / (n (n-1)) with F the sum of the
  convolution-kernel products over all (i, j) and L the leave-one-out kernel sum over j != i;
* ``loo_likelihood(bw, np.log)`` (cv_ml, SM:kernel_density.py:126-160): -sum_i log L_i.

``CVObjective`` keeps the observations resident on the device and evaluates the per-observation sums
F_i, L_i with ``hbx_kde_cv_terms`` (one workgroup per observation, the reference's per-dim kernels,
dim-ordered product and numpy's pairwise summation order).  The host keeps what is O(n) or O(D): the
continuous bandwidth product (a sequential np.prod), the in-order sums over i (np.cumsum is the same
left-to-right accumulation as the reference's ``F += k_bar_sum`` loop), the log of cv_ml, and the
Nelder-Mead search itself (the same scipy routine the reference calls).  There is no CPU path: every
objective evaluation runs the HIP kernel.
"""

import numpy as np

from . import _native as N
from .kde import bandwidth_factor, default_device, var_type_codes

C2 = 1. / np.sqrt(2 * np.pi)  # SM:kernels.py gaussian
C4 = 1. / np.sqrt(4 * np.pi)  # SM:kernels.py gaussian_convolution


def _torch():
    import torch
    return torch


def level_tables(data, var_type):
    """Per categorical dim: the ascending unique values of -X[:, d] (the order of np.unique(Xi) in
    aitchison_aitken_convolution, SM:kernels.py:166-174, over imse's negated data) and, per row i, the
    level count of the column without row i (np.unique(-X_not_i[:, d]).size, SM:kernels.py:59-60)."""
    n, D = data.shape
    lev, off = [], [0]
    loo = np.zeros((n, D), dtype=np.int32)
    for d, t in enumerate(var_type):
        if t == "c":
            off.append(off[-1])
            continue
        vals, inv, cnt = np.unique(-data[:, d], return_inverse=True, return_counts=True)
        lev.extend(vals.tolist())
        off.append(off[-1] + vals.size)
        loo[:, d] = vals.size - (cnt[inv.reshape(-1)] == 1)
    return np.array(lev if lev else [0.0], dtype=np.float64), np.array(off, dtype=np.int32), loo


class CVObjective(object):
    """The two CV objectives of one data set, resident on the GPU.

    ``imse(bw)`` and ``loo_likelihood(bw)`` return the same values as statsmodels'
    ``KDEMultivariate.imse`` / ``.loo_likelihood(bw, np.log)`` (to the last ulp or two of exp/log).
    """

    def __init__(self, data, var_type, device=None, stream=None):
        torch = _torch()
        data = np.ascontiguousarray(np.asarray(data, dtype=np.float64))
        if data.ndim != 2 or data.shape[1] != len(var_type):
            raise ValueError("data must be [nobs, len(var_type)]")
        if any(t not in "cu" for t in var_type):
            raise ValueError("var_type: only 'c' and 'u' are used by the generators (got %r)" % var_type)
        n, D = data.shape
        if n <= D:  # SM:kernel_density.py:107-109
            raise ValueError("The number of observations must be larger than the number of variables.")
        if D > int(N.lib().hbx_max_dims()):
            raise ValueError("at most %d dims" % int(N.lib().hbx_max_dims()))
        self.device = device if device is not None else default_device()
        self.stream = stream
        self.var_type = var_type
        self.data = data
        self.nobs, self.k_vars = n, D
        self.iscont = np.array([t == "c" for t in var_type])
        lev, off, loo = level_tables(data, var_type)
        t = lambda a: torch.from_numpy(a).to(self.device)  # noqa: E731
        self.X_dev = t(data)
        self.vt_dev = t(var_type_codes(var_type))
        self.lev_dev, self.off_dev, self.loo_dev = t(lev), t(off), t(loo)
        self.bw_dev = torch.empty(D, dtype=torch.float64, device=self.device)
        self.F_dev = torch.empty(n, dtype=torch.float64, device=self.device)
        self.L_dev = torch.empty(n, dtype=torch.float64, device=self.device)
        self.evals = 0

    def terms(self, bw, want_F=True, want_L=True):
        """(F[n], L[n]) per-observation sums at bandwidths bw (host numpy arrays; None if not asked)."""
        torch = _torch()
        bw = np.ascontiguousarray(np.asarray(bw, dtype=np.float64).reshape(-1))
        if bw.size != self.k_vars:
            raise ValueError("bw must have %d entries" % self.k_vars)
        bwprod = float(bw[self.iscont].prod())  # sequential np.prod, as imse/gpke
        with torch.cuda.stream(self.stream) if self.stream is not None else _null():
            self.bw_dev.copy_(torch.from_numpy(bw), non_blocking=False)
            F = self.F_dev if want_F else None
            L = self.L_dev if want_L else None
            N.call("hbx_kde_cv_terms", N.ptr(self.X_dev), self.nobs, self.k_vars, N.ptr(self.vt_dev),
                   N.ptr(self.bw_dev), N.ptr(self.lev_dev), N.ptr(self.off_dev), N.ptr(self.loo_dev), C4, C2,
                   bwprod, N.ptr(F), N.ptr(L), N.stream_handle(self.stream))
            out = (F.cpu().numpy() if want_F else None, L.cpu().numpy() if want_L else None)
        self.evals += 1
        return out

    def imse(self, bw):
        """SM:kernel_density.py:246-332 (bw='cv_ls' objective)."""
        F, L = self.terms(bw)
        n = self.nobs
        Fs = float(np.cumsum(F)[-1])  # F = 0; F += k_bar_sum, in row order
        Ls = float(np.cumsum(L)[-1])
        return Fs / n ** 2 - 2 * Ls / (n * (n - 1))

    def loo_likelihood(self, bw, func=np.log):
        """SM:kernel_density.py:126-160 (bw='cv_ml' objective with func=np.log): -sum_i func(L_i)."""
        _, L = self.terms(bw, want_F=False)
        with np.errstate(divide="ignore", invalid="ignore"):
            v = func(L)
        return -float(np.cumsum(v)[-1])

    def normal_reference(self):
        """SM:_kernel_base.py:250-265: 1.06 std(X, axis=0) n^(-1/(4+q)) (host, O(n D), once)."""
        return 1.06 * np.std(self.data, axis=0) * bandwidth_factor(self.nobs, self.k_vars)

    def set_bw_bounds(self, bw):
        """SM:_kernel_base.py:267-277."""
        bw = np.array(bw, dtype=np.float64)
        bw[bw < 0] = 1e-10
        bw[~self.iscont] = np.minimum(bw[~self.iscont], 1.)
        return bw

    def select(self, method="cv_ls", x0=None):
        """SM:_kernel_base.py:279-332: Nelder-Mead (scipy.optimize.fmin, maxiter=maxfun=1000, xtol=1e-3)
        from the normal-reference bandwidths, then the bounds."""
        from scipy import optimize
        if method == "cv_ls":
            fun, args = self.imse, ()
        elif method == "cv_ml":
            fun, args = self.loo_likelihood, (np.log,)
        else:
            raise ValueError("method must be 'cv_ls' or 'cv_ml'")
        h0 = self.normal_reference() if x0 is None else np.asarray(x0, dtype=np.float64)
        bw = optimize.fmin(fun, x0=h0, args=args, maxiter=1e3, maxfun=1e3, disp=0, xtol=1e-3)
        return self.set_bw_bounds(bw)


class _null(object):
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def select_bandwidth(data, var_type, bw="cv_ls", device=None):
    """Bandwidths KDEMultivariate(data, var_type, bw=...) would choose (SM:_kernel_base.py:103-139):
    'normal_reference', 'cv_ls', 'cv_ml' or an explicit array."""
    if not isinstance(bw, str):
        return np.asarray(bw, dtype=np.float64)
    data = np.asarray(data, dtype=np.float64)
    if bw == "normal_reference":
        return 1.06 * np.std(data, axis=0) * bandwidth_factor(data.shape[0], data.shape[1])
    return CVObjective(data, var_type, device=device).select(bw)


__all__ = ["CVObjective", "select_bandwidth", "level_tables"]
