"""The reference's arithmetic under THIS process's numpy, for near ties (``ties='process'``).

The GPU re-scores every shortlisted candidate in fp64 with statsmodels' operation order and numpy
1.26.4's exp restated bit for bit (the pinned reference).  Other numpy builds' exp differ by ulps
(numpy 2.2 in ~23 % of outputs), so a near tie may be ordered differently by the reference run on
another numpy; each exact score carries the relative spread that can cause (``AcqResult.rel``).  On
request, candidates within that spread of the winner (flag ``HBX_ACQ_NEAR_TIE``) are re-ordered here,
on the host, with the very numpy expressions the reference evaluates -- KDEMultivariate.pdf (statsmodels 0.12.2 kernel_density.py:162-196) -> gpke
(_kernel_base.py:456-518) -> gaussian / aitchison_aitken (kernels.py:108-125, 23-65) -- and BOHB's
``max(1e-8, g) / max(l, 1e-8)`` with a strict ``<`` over the candidates in index order
(bohb.py:129, 149-152).  This is part of the engine (a few candidates, a few numpy calls each), not
a fallback: by default the GPU's pinned-reference pick is final.  The KDEs' rows are in the
reference's order even where losses tie (the refit's argsort is numpy's, hbx_npsort.h), so these
expressions see the reference's very arrays.
"""

import warnings

import numpy as np

CLAMP = 1e-8  # bohb.py:129


def kde_pdf(data, bw, var_type, nlev, x):
    """pdf of one point, numpy expressions in the reference's order (bit-identical to
    KDEMultivariate.pdf on the same numpy).  ``nlev``: observed levels per categorical dim
    (np.unique(data[:, d]).size, what aitchison_aitken computes when num_levels is None)."""
    data = np.asarray(data, dtype=np.float64)
    x = np.asarray(x, dtype=np.float64).reshape(-1)
    bw = np.asarray(bw, dtype=np.float64)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        Kval = np.empty(data.shape)
        for ii, vtype in enumerate(var_type):
            Xi = data[:, ii]
            h = bw[ii]
            if vtype == "c":
                Kval[:, ii] = (1. / np.sqrt(2 * np.pi)) * np.exp(-(Xi - x[ii]) ** 2 / (h ** 2 * 2.))
            else:
                Xi = Xi.reshape(Xi.size)
                kernel_value = np.ones(Xi.size) * h / (np.asarray(nlev[ii]) - 1)
                idx = Xi == x[ii]
                kernel_value[idx] = (idx * (1 - h))[idx]
                Kval[:, ii] = kernel_value
        iscontinuous = np.array([c == "c" for c in var_type])
        dens = Kval.prod(axis=1) / np.prod(bw[iscontinuous])
        return dens.sum(axis=0) / data.shape[0]


def bohb_score(l, g):
    """bohb.py:129 with Python max() semantics (NaN g -> 1e-8, NaN l -> NaN)."""
    return max(CLAMP, g) / max(l, CLAMP)


def resolve(good, bad, rows, indices):
    """Among candidates ``indices`` (rows[k] = the candidate's coordinates), the reference's pick:
    strict '<' in index order against best = +inf.  good/bad: objects with .data, .bw, .var_type,
    .nlev (DeviceKDE).  Returns (index, score, pdf_l, pdf_g) or None when no score is finite."""
    order = np.argsort(np.asarray(indices), kind="stable")
    best, pick = np.inf, None
    for k in order:
        l = float(kde_pdf(good.data, good.bw, good.var_type, good.nlev, rows[k]))
        g = float(kde_pdf(bad.data, bad.bw, bad.var_type, bad.nlev, rows[k]))
        s = bohb_score(l, g)
        if s < best:
            best, pick = s, (int(indices[k]), s, l, g)
    return pick
