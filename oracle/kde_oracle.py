"""ORACLE -- test infrastructure only.

CPU restatement (numpy, fp64) of the reference arithmetic on the KDE acquisition and
successive-halving promotion path.  It is imported ONLY by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg, always as the checker,
never as the thing measured or shipped.  The engine (``hpbandster_amd``) never imports it
and fails loudly when its HIP library is missing.

Pinning: every function here is checked against golden fixtures generated from the
reference itself (``tests/golden/gen_golden.py`` runs the reference's ``bohb.py`` /
``HB_iteration.py`` / ``HB_master.py`` on top of statsmodels 0.12.2, the third-party library
holding BOHB's KDE arithmetic, pinned by the oracle interpreter /opt/conda/bin/python3.9).
See ``tests/test_oracle_golden.py``.

Citations: ``path:line`` = reference file under /root/reference; ``SM:`` =
statsmodels 0.12.2 ``statsmodels/nonparametric/`` (not vendored by the reference).
"""

import math

import numpy as np

from oracle import np_argsort

CLAMP = 1e-8  # bohb.py:129


# --------------------------------------------------------------------------------------
# KDE fit (BOHB.new_result -> KDEMultivariate(..., bw='normal_reference'))


def bohb_split_sizes(n, min_points, top_n_percent=15):
    """bohb.py:224-225 (integer floor division)."""
    n_good = max(min_points, (top_n_percent * n) // 100)
    n_bad = max(min_points, ((100 - top_n_percent) * n) // 100)
    return n_good, n_bad


def bohb_split(X, losses, min_points, top_n_percent=15):
    """bohb.py:220-237: argsort the losses, good = head, bad = tail (may overlap).

    Returns (good_rows, bad_rows) or None when the reference returns without refitting
    (too few rows, bohb.py:216-217, or rows <= dims, bohb.py:234-237).
    """
    n, D = X.shape
    if n <= min_points + 1:
        return None
    n_good, n_bad = bohb_split_sizes(n, min_points, top_n_percent)
    idx = np_argsort.argsort(losses)  # numpy 1.26.4's unstable order, ties included
    good, bad = idx[:n_good], idx[-n_bad:]
    if good.shape[0] <= D or bad.shape[0] <= D:
        return None
    return good, bad


def normal_reference_bw(data):
    """SM:_kernel_base.py:250-265: 1.06 * std(X, axis=0) * n**(-1/(4+q)), for every dim."""
    X = np.std(data, axis=0)
    return 1.06 * X * data.shape[0] ** (-1. / (4 + data.shape[1]))


def num_levels(data, var_type):
    """SM:kernels.py:59-60: observed level count np.unique(column).size, per 'u' column."""
    return np.array([np.unique(data[:, d]).size if t == "u" else 0 for d, t in enumerate(var_type)])


# --------------------------------------------------------------------------------------
# pdf (KDEMultivariate.pdf -> gpke), reference operation order


def _gaussian(h, Xi, x):
    """SM:kernels.py:108-125."""
    return (1. / np.sqrt(2 * np.pi)) * np.exp(-(Xi - x) ** 2 / (h ** 2 * 2.))


def _aitchison_aitken(h, Xi, x, nlev):
    """SM:kernels.py:23-65 with num_levels taken from the KDE's own data column."""
    kernel_value = np.ones(Xi.size) * h / (nlev - 1)
    idx = Xi == x
    kernel_value[idx] = (idx * (1 - h))[idx]
    return kernel_value


def pdf(data, bw, var_type, x, nlev=None):
    """KDEMultivariate.pdf for one point (SM:kernel_density.py:162-196, SM:_kernel_base.py:456-518).

    Kval[:, d] per dim, row product / prod(bw[continuous]), contiguous sum, / nobs.
    Bit-identical to statsmodels on the same numpy (verified against the golden fixtures).
    """
    data = np.asarray(data, dtype=np.float64)
    x = np.asarray(x, dtype=np.float64).reshape(-1)
    if nlev is None:
        nlev = num_levels(data, var_type)
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        Kval = np.empty(data.shape)
        for ii, vt in enumerate(var_type):
            if vt == "c":
                Kval[:, ii] = _gaussian(bw[ii], data[:, ii], x[ii])
            else:
                Kval[:, ii] = _aitchison_aitken(bw[ii], data[:, ii], x[ii], np.asarray(nlev[ii]))
        iscont = np.array([c == "c" for c in var_type])
        dens = Kval.prod(axis=1) / np.prod(bw[iscont])
        return dens.sum(axis=0) / data.shape[0]


def pdf_many(data, bw, var_type, X, nlev=None):
    if nlev is None:
        nlev = num_levels(np.asarray(data), var_type)
    return np.array([pdf(data, bw, var_type, x, nlev) for x in np.asarray(X)])


def log_pdf_many(data, bw, var_type, X, nlev=None):
    """Natural-log densities in fp64 log space (no underflow), for tolerance checks.

    NaN where the reference pdf is NaN; -inf where the pdf is <= 0.
    """
    data = np.asarray(data, dtype=np.float64)
    n, D = data.shape
    if nlev is None:
        nlev = num_levels(data, var_type)
    bw = np.asarray(bw, dtype=np.float64)
    out = np.empty(len(X))
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for i, x in enumerate(np.asarray(X, dtype=np.float64)):
            logk = np.zeros(n)
            sign = np.ones(n)
            nan = False
            for d, vt in enumerate(var_type):
                if vt == "c":
                    if bw[d] == 0:
                        nan = True
                        break
                    logk += -0.5 * math.log(2 * math.pi) - (data[:, d] - x[d]) ** 2 / (2 * bw[d] ** 2)
                else:
                    a = 1 - bw[d]
                    if nlev[d] == 1:  # h == 0: match -> 1, mismatch -> 0/0
                        if np.any(data[:, d] != x[d]):
                            nan = True
                            break
                        continue
                    b = bw[d] / (nlev[d] - 1)
                    m = data[:, d] == x[d]
                    with np.errstate(divide="ignore"):
                        logk += np.where(m, np.log(abs(a)), np.log(b))
                    sign *= np.where(m & (a < 0), -1.0, 1.0)
            if nan:
                out[i] = np.nan
                continue
            mx = np.max(logk)
            if not np.isfinite(mx):
                out[i] = -np.inf
                continue
            s = np.sum(sign * np.exp(logk - mx))
            norm = -math.log(n) - sum(math.log(bw[d]) for d, vt in enumerate(var_type) if vt == "c")
            out[i] = (mx + math.log(s) + norm) if s > 0 else -np.inf
    return out


# --------------------------------------------------------------------------------------
# BOHB selection (bohb.py:129, 149-152)


def py_score(l, g):
    """max(1e-8, g) / max(l, 1e-8) with Python max() semantics (NaN g -> 1e-8, NaN l -> NaN)."""
    return max(CLAMP, g) / max(l, CLAMP)


def py_argmin(scores):
    """Strict '<' against best=+inf: first index of the minimum over non-NaN, non-inf scores."""
    best, best_i = np.inf, -1
    for i, v in enumerate(scores):
        if v < best:
            best, best_i = v, i
    return best_i


def select(pdf_l, pdf_g):
    scores = np.array([py_score(float(l), float(g)) for l, g in zip(pdf_l, pdf_g)])
    return py_argmin(scores), scores


# --------------------------------------------------------------------------------------
# successive halving promotion (HB_iteration.py:179-182, 239-242)


def sh_advance(losses, k, stable=False):
    """ranks = argsort(argsort(losses)); advance = ranks < k, over the REVIEW (finite) entries only.

    Non-finite losses are CRASHED in register_result (HB_iteration.py:102-106) and never ranked.
    Returns a bool mask over all entries.  Tied losses are ordered as numpy 1.26.4's default argsort
    orders them (np_argsort.py); ``stable=True`` ranks ties by position instead.
    """
    losses = np.asarray(losses, dtype=np.float64)
    ok = np.isfinite(losses)
    adv = np.zeros(losses.shape[0], dtype=bool)
    sub = losses[ok]
    inner = np.argsort(sub, kind="stable") if stable else np_argsort.argsort(sub)
    ranks = np.argsort(inner, kind="stable")  # a permutation: no ties
    adv[np.nonzero(ok)[0]] = ranks < k
    return adv


# --------------------------------------------------------------------------------------
# Hyperband budgets and brackets (HB_master.py:93-94, 161-168)


def hb_budgets(eta, min_budget, max_budget):
    max_SH_iter = -int(np.log(min_budget / max_budget) / np.log(eta)) + 1
    budgets = max_budget * np.power(eta, -np.linspace(max_SH_iter - 1, 0, max_SH_iter))
    return max_SH_iter, budgets


def hb_bracket(it, eta, max_SH_iter):
    s = max_SH_iter - 1 - (it % max_SH_iter)
    n0 = int(np.floor((max_SH_iter) / (s + 1)) * eta ** s)
    ns = [max(int(n0 * (eta ** (-i))), 1) for i in range(s + 1)]
    return s, ns


# --------------------------------------------------------------------------------------
# cross-validation bandwidth objectives (KDEMultivariate bw='cv_ls' / 'cv_ml'; kde.py:145-147)


def _gaussian_convolution(h, Xi, x):
    """SM:kernels.py gaussian_convolution: (1/sqrt(4 pi)) exp(-(Xi - x)^2 / (h^2 4))."""
    return (1. / np.sqrt(4 * np.pi)) * np.exp(-(Xi - x) ** 2 / (h ** 2 * 4.))


def _aitchison_aitken_convolution(h, Xi, Xj):
    """SM:kernels.py:166-174: sum over the column's levels (np.unique order) of the two AA kernels."""
    vals = np.unique(Xi)
    c = vals.size
    out = np.zeros(Xi.size)
    for x in vals:
        out += _aitchison_aitken(h, Xi, x, np.asarray(c)) * _aitchison_aitken(h, np.asarray(Xj).reshape(1), x, np.asarray(c))
    return out


def _loo_rows(n, i):
    m = np.ones(n, dtype=bool)
    m[i] = False
    return m


def cv_terms(data, bw, var_type, rows=None):
    """Per-observation sums of the two CV objectives, reference operation order.

    F[i] = convolution-kernel sum over all j (SM:kernel_density.py:300-311, imse's first loop),
    L[i] = leave-one-out kernel sum over j != i (SM:kernel_density.py:313-322 == the gpke call of
    loo_likelihood, SM:kernel_density.py:153-158); both divided by the continuous bandwidth product
    (a sequential np.prod) before numpy's contiguous sum.  ``rows``: only these i (others NaN).
    """
    data = np.asarray(data, dtype=np.float64)
    bw = np.asarray(bw, dtype=np.float64)
    n, D = data.shape
    neg = -data
    iscont = np.array([t == "c" for t in var_type])
    bwprod = bw[iscont].prod()
    F = np.full(n, np.nan)
    L = np.full(n, np.nan)
    rows = range(n) if rows is None else rows
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        K = np.empty((n, D))
        for i in rows:
            for d, t in enumerate(var_type):
                if t == "c":
                    K[:, d] = _gaussian_convolution(bw[d], neg[:, d], neg[i, d])
                else:
                    K[:, d] = _aitchison_aitken_convolution(bw[d], neg[:, d], neg[i, d])
            F[i] = (K.prod(axis=1) / bwprod).sum(axis=0)
        K = np.empty((n - 1, D))
        for i in rows:
            Xn = -data[_loo_rows(n, i)]
            for d, t in enumerate(var_type):
                if t == "c":
                    K[:, d] = _gaussian(bw[d], Xn[:, d], neg[i, d])
                else:
                    K[:, d] = _aitchison_aitken(bw[d], Xn[:, d], neg[i, d], np.asarray(np.unique(Xn[:, d]).size))
            L[i] = (K.prod(axis=1) / bwprod).sum(axis=0)
    return F, L


def imse_from_terms(F, L, n):
    """SM:kernel_density.py:300-326: F and L accumulated from int 0 in row order, then the CV formula."""
    Fs, Ls = 0, 0
    for v in F:
        Fs += v
    for v in L:
        Ls += v
    return Fs / n ** 2 - 2 * Ls / (n * (n - 1))


def loo_from_terms(L):
    """SM:kernel_density.py:153-160 with func=np.log: -(sum_i log L_i), accumulated from int 0."""
    s = 0
    with np.errstate(divide="ignore", invalid="ignore"):
        for v in L:
            s += np.log(v)
    return -s


def imse(data, bw, var_type):
    F, L = cv_terms(data, bw, var_type)
    return imse_from_terms(F, L, np.asarray(data).shape[0])


def loo_likelihood(data, bw, var_type):
    _, L = cv_terms(data, bw, var_type)
    return loo_from_terms(L)


def set_bw_bounds(bw, var_type):
    """SM:_kernel_base.py:267-277: negative -> 1e-10, categorical capped at 1."""
    bw = np.array(bw, dtype=np.float64)
    bw[bw < 0] = 1e-10
    cat = np.array([t != "c" for t in var_type])
    bw[cat] = np.minimum(bw[cat], 1.)
    return bw


def cv_bandwidth(data, var_type, method="cv_ls"):
    """SM:_kernel_base.py:279-332: scipy.optimize.fmin (Nelder-Mead) from the normal-reference rule."""
    from scipy import optimize
    data = np.asarray(data, dtype=np.float64)
    h0 = normal_reference_bw(data)
    if method == "cv_ls":
        obj = lambda b: imse(data, b, var_type)  # noqa: E731
    elif method == "cv_ml":
        obj = lambda b: loo_likelihood(data, b, var_type)  # noqa: E731
    else:
        raise ValueError(method)
    bw = optimize.fmin(obj, x0=h0, maxiter=1e3, maxfun=1e3, disp=0, xtol=1e-3)
    return set_bw_bounds(bw, var_type)
