#!/opt/conda/bin/python3.9 -B
"""Golden vectors for the cross-validation bandwidth objectives.

    PYTHONDONTWRITEBYTECODE=1 /opt/conda/bin/python3.9 -B tests/golden/gen_cv.py

Runs statsmodels 0.12.2 (the library the reference's KernelDensityEstimator calls, kde.py:145-147)
in the container's oracle interpreter: KDEMultivariate.imse and .loo_likelihood(bw, np.log) at a few
bandwidth vectors, and the bandwidths bw='cv_ls' / bw='cv_ml' select (Nelder-Mead from the normal
reference rule).  Writes tests/golden/cv_<case>.npz.  Data only: inputs and statsmodels' outputs.
"""
import os
import time

import numpy as np
import scipy
import statsmodels
from statsmodels.nonparametric.kernel_density import KDEMultivariate

HERE = os.path.dirname(os.path.abspath(__file__))


def case(name, X, var_type, seed):
    rs = np.random.RandomState(seed)
    kde = KDEMultivariate(X, var_type=var_type, bw="normal_reference")
    h0 = kde.bw.copy()
    pts = [h0, h0 * 0.5, h0 * 0.8, h0 * 1.3, h0 * (0.6 + rs.rand(len(h0)))]
    cat = np.array([t == "u" for t in var_type])
    for p in pts:
        p[cat] = np.minimum(p[cat], 0.9)  # Aitchison-Aitken lambda stays in [0, 1)
    pts = np.array(pts)
    imse = np.array([kde.imse(p) for p in pts])
    loo = np.array([kde.loo_likelihood(p, np.log) for p in pts])
    t0 = time.time()
    bw_ls = KDEMultivariate(X, var_type=var_type, bw="cv_ls").bw
    t_ls = time.time() - t0
    t0 = time.time()
    bw_ml = KDEMultivariate(X, var_type=var_type, bw="cv_ml").bw
    t_ml = time.time() - t0
    np.savez(os.path.join(HERE, "cv_%s.npz" % name), X=X, var_type=np.array(var_type), bw_points=pts, imse=imse,
             loo=loo, h0=h0, bw_cv_ls=bw_ls, bw_cv_ml=bw_ml, seconds_cv_ls=t_ls, seconds_cv_ml=t_ml,
             versions=np.array([statsmodels.__version__, scipy.__version__, np.__version__]))
    print("%s: n=%d D=%d  cv_ls %.1fs %s  cv_ml %.1fs %s" % (name, X.shape[0], X.shape[1], t_ls, bw_ls, t_ml, bw_ml))


def main():
    rs = np.random.RandomState(11)
    case("c3", rs.rand(60, 3), "ccc", 1)
    rs = np.random.RandomState(12)
    n = 80
    X = np.column_stack([rs.rand(n), rs.rand(n), rs.randint(0, 3, n), rs.randint(0, 3, n)]).astype(float)
    X[17, 3] = 3.0  # a level seen once: its leave-one-out column has one level fewer
    case("mixed", X, "ccuu", 2)
    rs = np.random.RandomState(13)
    case("c6", rs.rand(300, 6), "cccccc", 3)


if __name__ == "__main__":
    main()
