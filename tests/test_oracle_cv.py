"""The CPU restatement of the CV bandwidth objectives (oracle/kde_oracle.py cv_terms / imse /
loo_likelihood / cv_bandwidth) against statsmodels 0.12.2's own outputs (tests/golden/cv_*.npz,
written by tests/golden/gen_cv.py), and the host-side level tables of hpbandster_amd.cv.

Tolerance: objectives within 1e-14 relative (numpy's exp differs by an ulp between the fixture's
numpy 1.26 and this numpy); selected bandwidths within 1e-9 relative (same Nelder-Mead path).
"""
import numpy as np
import pytest

from oracle import kde_oracle as O

CASES = ["c3", "mixed", "c6"]


def load(name):
    import os
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "cv_%s.npz" % name))
    return {k: d[k] for k in d.files}


@pytest.mark.parametrize("name", CASES)
def test_objectives_match_statsmodels(name):
    c = load(name)
    vt = str(c["var_type"])
    for p, im, lo in zip(c["bw_points"], c["imse"], c["loo"]):
        F, L = O.cv_terms(c["X"], p, vt)
        n = c["X"].shape[0]
        np.testing.assert_allclose(O.imse_from_terms(F, L, n), im, rtol=1e-14)
        np.testing.assert_allclose(O.loo_from_terms(L), lo, rtol=1e-14)


def test_normal_reference_start_matches():
    for name in CASES:
        c = load(name)
        np.testing.assert_array_equal(O.normal_reference_bw(c["X"]), c["h0"])


@pytest.mark.parametrize("name", ["c3", "mixed"])
@pytest.mark.parametrize("method", ["cv_ls", "cv_ml"])
def test_bandwidth_selection_matches_statsmodels(name, method):
    c = load(name)
    bw = O.cv_bandwidth(c["X"], str(c["var_type"]), method)
    np.testing.assert_allclose(bw, c["bw_" + method], rtol=1e-9)


def test_cv_terms_rows_subset():
    c = load("mixed")
    vt = str(c["var_type"])
    F, L = O.cv_terms(c["X"], c["h0"], vt)
    F2, L2 = O.cv_terms(c["X"], c["h0"], vt, rows=[0, 17, 79])
    np.testing.assert_array_equal(F2[[0, 17, 79]], F[[0, 17, 79]])
    np.testing.assert_array_equal(L2[[0, 17, 79]], L[[0, 17, 79]])
    assert np.isnan(F2[1]) and np.isnan(L2[1])


def test_level_tables_match_leave_one_out_unique():
    from hpbandster_amd.cv import level_tables
    c = load("mixed")
    X = c["X"]
    lev, off, loo = level_tables(X, "ccuu")
    assert list(off) == [0, 0, 0, 3, 7]
    np.testing.assert_array_equal(lev[0:3], np.unique(-X[:, 2]))
    np.testing.assert_array_equal(lev[3:7], np.unique(-X[:, 3]))
    n = X.shape[0]
    for i in range(n):
        m = np.ones(n, bool)
        m[i] = False
        for d in (2, 3):
            assert loo[i, d] == np.unique(-X[m, d]).size
    assert loo[17, 3] == 3 and loo[0, 3] == 4
